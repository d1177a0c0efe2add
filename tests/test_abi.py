"""The C-ABI library loads and exports every entry point include/miner_score.h declares; host-only
entry points answer without a device. No compute call is made (runs on CPU-only machines)."""
import ctypes
import os
import re

import pytest
import torch

from miner_amd import _lib, ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include")))
           if h.endswith(".h")]


def declared_symbols():
    names = set()
    for path in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
        names |= set(re.findall(r"\b(miner_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        from miner_amd.build import build_library
        build_library()
    return _lib.lib()


def test_header_and_binding_agree():
    decl = declared_symbols()
    assert decl == sorted(_lib.SIGNATURES), (decl, sorted(_lib.SIGNATURES))


def test_every_declared_symbol_is_exported(lib):
    for name in declared_symbols():
        assert hasattr(lib, name), name
    # the exports are plain C symbols (no C++ mangling)
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_symbols():
        assert ctypes.cast(getattr(raw, name), ctypes.c_void_p).value


def test_abi_version(lib):
    assert lib.miner_abi_version() == _lib.ABI_VERSION


def test_supported_shapes(lib):
    F32, BF16 = _lib.DTYPE_F32, _lib.DTYPE_BF16
    for dt in (F32, BF16):
        assert lib.miner_supported(dt, 50, 768, 200, 32) == 0      # config 3 (MIND-large)
        assert lib.miner_supported(dt, 50, 256, 200, 32) == 0      # config 2 (MIND-small)
    assert lib.miner_supported(F32, 20, 64, 32, 4) == 0            # config 1 (demo)
    assert lib.miner_supported(F32, 50, 100, 200, 32) != 0          # d % 32
    assert lib.miner_supported(F32, 50, 768, 200, 64) != 0          # K > 32
    assert lib.miner_supported(F32, 200, 768, 200, 32) != 0         # L > 64
    assert lib.miner_supported(7, 50, 768, 200, 32) == -1           # bad dtype -> EINVAL


def test_wide_path_shapes(lib):
    """Past the fused kernel (K > 32 or L > 64) the wide path takes K <= 64, L <= 256, Dc <= 256,
    d <= 768 (include/miner_wide.h); the host routing (ops._fused_or_wide) follows these answers."""
    F32, BF16 = _lib.DTYPE_F32, _lib.DTYPE_BF16
    assert lib.miner_wide_supported(F32, 120, 256, 64, 64) == 0
    assert lib.miner_wide_supported(BF16, 200, 768, 200, 64) == 0       # config-5 user dims
    assert lib.miner_wide_supported(F32, 257, 256, 64, 32) == -2        # L > 256
    assert lib.miner_wide_supported(F32, 50, 256, 64, 65) == -2         # K > 64
    assert lib.miner_wide_supported(F32, 50, 1024, 64, 32) == -2        # d > 768
    assert lib.miner_wide_supported(BF16, 50, 96, 64, 32) == -2         # 16-bit: d % 64
    assert lib.miner_wide_supported(F32, 50, 96, 64, 32) == 0
    assert lib.miner_wide_supported(9, 50, 256, 64, 32) == -1
    with pytest.raises(ValueError, match="wide path"):
        ops._fused_or_wide(F32, 300, 256, 64, 32)
    assert ops._fused_or_wide(F32, 50, 256, 64, 32) is True
    assert ops._fused_or_wide(F32, 120, 256, 64, 64) is False


def test_wide_argument_errors_before_any_launch(lib):
    P = ctypes.c_void_p(16)
    assert lib.miner_score_wide(None, 0, 7, P, P, P, None, 0, None, None, 1, 4, 256, 64, P) == -1   # score type
    assert lib.miner_score_wide(None, 0, 0, P, None, P, None, 0, None, None, 1, 4, 256, 64, P) == -1  # no proj
    assert lib.miner_score_wide(None, 0, 1, P, None, P, None, 0, None, None, 1, 4, 256, 65, P) == -2  # K > 64
    assert lib.miner_score_wide(None, 0, 1, P, None, P, None, 0, None, P, 1, 4, 256, 8, P) == -1     # value: weighted
    assert lib.miner_score_wide(None, 0, 1, P, None, P, None, 0, None, None, 0, 4, 256, 8, P) == 0   # B = 0: no launch
    assert lib.miner_wide_proj(None, 0, P, P, 4, 96, P) == -2                                       # d % 64
    assert lib.miner_wide_proj(None, 0, None, P, 4, 128, P) == -1


def test_lds_fits_one_cu(lib):
    for dt in (_lib.DTYPE_F32, _lib.DTYPE_BF16):
        for st in (0, 1, 2, 3):
            n = lib.miner_lds_bytes(dt, st, 50, 768, 200)
            assert 0 < n <= 160 * 1024, (dt, st, n)


def test_packed_bytes(lib):
    assert lib.miner_packed_weights_bytes(_lib.DTYPE_BF16, 768, 200, 32) > 2 * (768 * 768 + 200 * 768)
    # fp32: the bf16 layout's tiles at 4 bytes, then the fp16-pair copies of W2 and W1 (same bytes as
    # their fp32 tiles) and their row units (d, and Dc padded to 32-row tiles)
    w1, w2 = 7 * 24 * 1024, 24 * 24 * 1024
    assert lib.miner_packed_weights_bytes(_lib.DTYPE_F32, 768, 200, 32) == \
        2 * lib.miner_packed_weights_bytes(_lib.DTYPE_BF16, 768, 200, 32) + 4 * (w2 + 768 + w1 + 7 * 32)
    assert lib.miner_packed_weights_bytes(_lib.DTYPE_F32, 100, 200, 32) == 0


def test_argument_errors_before_any_launch(lib):
    # NULL pointers / bad enums are rejected on the host with the documented codes
    assert lib.miner_pack_weights(None, _lib.DTYPE_BF16, None, None, None, 768, 200, 32, None) == -1
    assert lib.miner_pack_weights(None, 5, None, None, None, 768, 200, 32, None) == -1
    assert lib.miner_score(None, _lib.DTYPE_BF16, 9, None, None, None, None, None, None,
                           1, 50, 40, 768, 200, 32, None, None) == -1
    assert lib.miner_score(None, _lib.DTYPE_BF16, 0, None, None, None, None, None, None,
                           1, 50, 40, 768, 200, 32, None, None) == -1
    for code in (0, -1, -2, -3, -4):
        assert lib.miner_strerror(code)


def test_product_path_has_no_cpu_fallback():
    x = torch.zeros((2, 4, 64))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.score(x, torch.ones((2, 4), dtype=torch.bool), torch.zeros((2, 3, 64)), torch.zeros((32, 64)),
                  torch.zeros((4, 32)), torch.zeros((64, 64)))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.pack_weights(torch.zeros((32, 64)), torch.zeros((4, 32)))


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "absent.so"))
    with pytest.raises(_lib.MinerLibraryError, match="no CPU fallback"):
        _lib.lib()
