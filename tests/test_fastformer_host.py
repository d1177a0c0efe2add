"""Host side of the FastFormer path (no GPU): parameter naming / flat-blob order against the
reference's state_dict (fixtures), C-ABI argument checks that return before any launch."""
import ctypes
import os

import numpy as np
import pytest
import torch

from miner_amd import _lib
from miner_amd import fastformer as ff
from miner_amd import synthetic

HERE = os.path.dirname(os.path.abspath(__file__))


def test_params_follow_reference_state_dict_order():
    z = np.load(os.path.join(HERE, "golden", "fastformer_cfg4_slice.npz"), allow_pickle=False)
    ref = [(k[2:], tuple(z[k].shape)) for k in z.files if k.startswith("p.")]
    assert ref == [(n, tuple(s)) for n, s in ff.PARAMS]


def test_dropin_module_parameter_names():
    enc = ff.FastformerEncoder()
    sd = enc.state_dict()
    assert [(k, tuple(v.shape)) for k, v in sd.items()] == [(n, tuple(s)) for n, s in ff.PARAMS]
    blob = ff.flatten_params(sd)
    assert blob.numel() == ff.PARAM_FLOATS == 940097
    model = ff.FastFormer(news_encoder=type("E", (torch.nn.Module,), {"embed_dim": 256})(), score_type="weighted",
                          dropout=0.2)
    assert torch.equal(ff.flatten_params(model.state_dict()), ff.flatten_params(model.fast_attn.state_dict()))


def test_flatten_rejects_bad_state():
    sd = ff.FastformerEncoder().state_dict()
    bad = dict(sd)
    del bad["LayerNorm.bias"]
    with pytest.raises(KeyError):
        ff.flatten_params(bad)
    bad = dict(sd)
    bad["encoders.0.attention.self.query_att.weight"] = torch.zeros(8, 256)
    with pytest.raises(ValueError):
        ff.flatten_params(bad)


def test_unsupported_configs_rejected():
    class Cfg:
        hidden_size, num_attention_heads, intermediate_size, num_hidden_layers = 256, 8, 256, 2
    with pytest.raises(ValueError):
        ff.FastformerEncoder(Cfg())


def test_synthetic_params_blob():
    p = synthetic.fastformer_params(0)
    assert p.shape == (ff.PARAM_FLOATS,) and p.dtype == torch.float32
    assert torch.equal(p, synthetic.fastformer_params(0))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        from miner_amd.build import build_library
        build_library()
    return _lib.lib()


def test_abi_host_entry_points(lib):
    F32, BF16 = _lib.DTYPE_F32, _lib.DTYPE_BF16
    elems_t = 13 * 65536 + 4 * 8192
    fp = (29 * 256 + 65536) * 4
    assert lib.miner_fastformer_packed_bytes(F32) == elems_t * 4 + fp
    assert lib.miner_fastformer_packed_bytes(BF16) == elems_t * 2 + fp
    assert lib.miner_fastformer_packed_bytes(7) == 0
    assert lib.miner_fastformer_lds_bytes(BF16) <= 160 * 1024
    assert lib.miner_fastformer_lds_bytes(F32) <= 160 * 1024


def test_abi_argument_errors(lib):
    """Invalid arguments are rejected before anything is launched (fake non-null pointers)."""
    P = ctypes.c_void_p(16)
    f = lib.miner_fastformer_score
    assert f(None, 0, P, P, P, None, P, 4, 65, 3, P, None) == -2          # L > 64: ESHAPE
    assert f(None, 0, P, P, P, None, P, 4, 0, 3, P, None) == -1           # L = 0
    assert f(None, 9, P, P, P, None, P, 4, 50, 3, P, None) == -1          # bad dtype
    assert f(None, 0, P, None, P, None, P, 4, 50, 3, P, None) == -1       # null mask
    assert f(None, 0, P, P, P, None, P, 4, 50, 3, None, None) == -1       # no output
    assert f(None, 0, ctypes.c_void_p(18), P, P, None, P, 4, 50, 3, P, None) == -3   # misaligned
    assert f(None, 0, P, P, P, None, P, 0, 50, 3, P, None) == 0           # B = 0: nothing to do
    g = lib.miner_fastformer_score_gather
    assert g(None, 0, P, 0, P, P, P, None, P, 4, 50, 3, P, None) == -1    # n_news = 0
    assert g(None, 0, P, 10, P, P, None, None, P, 4, 50, 3, P, None) == -1  # scores without cand_ids
