"""ctypes binding of libminer_hip.so (declared in include/miner_score.h).

Loading is lazy so that the host-only parts of the package (evaluator, sharding, config parsing)
import on a machine without the library; every scoring entry point calls ``lib()``, which raises
loudly when the HIP library is missing — there is no CPU fallback in the product path.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MINER_HIP_LIB", os.path.join(_HERE, "libminer_hip.so"))

# enums of include/miner_score.h
DTYPE_F32, DTYPE_BF16, DTYPE_F16, DTYPE_F32_MFMA, DTYPE_F32_X6 = 0, 1, 2, 3, 4
SCORE_WEIGHTED, SCORE_MAX, SCORE_MEAN, SCORE_NONE = 0, 1, 2, 3
SCORE_TYPES = {"weighted": SCORE_WEIGHTED, "max": SCORE_MAX, "mean": SCORE_MEAN, "none": SCORE_NONE}
ABI_VERSION = 5

# every symbol include/*.h declares: name -> (restype, argtypes)
_P = ctypes.c_void_p
_I = ctypes.c_int
SIGNATURES = {
    "miner_packed_weights_bytes": (ctypes.c_size_t, [_I, _I, _I, _I]),
    "miner_pack_weights": (_I, [_P, _I, _P, _P, _P, _I, _I, _I, _P]),
    "miner_score": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P]),
    "miner_score_gather": (_I, [_P, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P]),
    "miner_target_aware": (_I, [_P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "miner_target_weights_bytes": (ctypes.c_size_t, [_I, _I]),
    "miner_pack_target_weights": (_I, [_P, _I, _P, _I, _P]),
    "miner_supported": (_I, [_I, _I, _I, _I, _I]),
    "miner_lds_bytes": (_I, [_I, _I, _I, _I, _I]),
    "miner_strerror": (ctypes.c_char_p, [_I]),
    "miner_abi_version": (_I, []),
    # include/miner_fastformer.h
    "miner_fastformer_packed_bytes": (ctypes.c_size_t, [_I]),
    "miner_fastformer_pack": (_I, [_P, _I, _P, _P]),
    "miner_fastformer_score": (_I, [_P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P]),
    "miner_fastformer_score_gather": (_I, [_P, _I, _P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P]),
    "miner_fastformer_lds_bytes": (_I, [_I]),
    # include/miner_corpus.h
    "miner_encoder_packed_bytes": (ctypes.c_size_t, [_I, _I, _I, _I]),
    "miner_encoder_pack": (_I, [_P, _I, _P, _P, _P, _I, _I, _I, _P]),
    "miner_encode_users": (_I, [_P, _I, _P, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "miner_rank_topk": (_I, [_P, _I, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "miner_rank_topk_workspace_bytes": (ctypes.c_size_t, [_I, _I]),
    "miner_rank_topk_split_recommended": (_I, [_I]),
    "miner_rank_topk_ws": (_I, [_P, _I, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, ctypes.c_size_t]),
    # include/miner_news.h
    "miner_news_precompute": (_I, [_P, _I, _P, _I, _P, _I, _I, _I, _P, _P]),
    "miner_score_news": (_I, [_P, _I, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "miner_news_supported": (_I, [_I, _I, _I, _I, _I]),
    "miner_news_split_x2": (_I, [_P, _P, _I, _I, _P, _P]),
    "miner_score_news_x2": (_I, [_P, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    # include/miner_wide.h
    "miner_score_wide": (_I, [_P, _I, _I, _P, _P, _P, _P, _I, _P, _P, _I, _I, _I, _I, _P]),
    "miner_wide_proj": (_I, [_P, _I, _P, _P, _I, _I, _P]),
    "miner_wide_supported": (_I, [_I, _I, _I, _I, _I]),
    # include/miner_metrics.h
    "miner_impression_metrics": (_I, [_P, _P, _P, _P, _I, _P, _I, _P, _P]),
    "miner_auc_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "miner_global_auc": (_I, [_P, _P, _P, ctypes.c_int64, _P, ctypes.c_size_t, _P]),
}

_lib = None


class MinerLibraryError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """The loaded library; raises MinerLibraryError if it is missing or ABI-incompatible."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MinerLibraryError(
            f"{LIB_PATH} not found: build it with `python -m miner_amd.build` "
            "(the MINER scoring path has no CPU fallback)")
    handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    if handle.miner_abi_version() != ABI_VERSION:
        raise MinerLibraryError(f"ABI mismatch: library {handle.miner_abi_version()} != {ABI_VERSION}")
    _lib = handle
    return _lib


def check(code: int, what: str) -> None:
    if code != 0:
        msg = lib().miner_strerror(code).decode()
        raise RuntimeError(f"{what} failed with code {code}: {msg}")
