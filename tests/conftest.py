import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    # single-class impressions are NaN by design (the reference nanmeans them, evaluation.py:59)
    config.addinivalue_line("filterwarnings", "ignore:Only one class is present in y_true")


def golden_names():
    """The MINER scoring fixtures (make_golden.py); reader_*.npz belong to the format tests and
    fastformer_*.npz / corpus_*.npz to the FastFormer / full-corpus tests."""
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))
                  if not os.path.basename(p).startswith(("reader_", "fastformer_", "corpus_")))


def news_golden_names():
    """The fixtures inside the news path's limits (L <= 64, K <= 32 with K % 4 == 0): the wide_*
    fixtures (K up to 64, L up to 120) go through the wide path instead (include/miner_wide.h)."""
    out = []
    for n in golden_names():
        z = np.load(os.path.join(GOLDEN_DIR, n + ".npz"), allow_pickle=False)
        if int(z["L"]) <= 64 and int(z["K"]) <= 32 and int(z["K"]) % 4 == 0:
            out.append(n)
    return out


def wide_golden_names():
    return [n for n in golden_names() if n.startswith("wide_")]


def load_golden(name):
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    g = {k: z[k] for k in z.files}
    for k in ("B", "L", "K", "d", "Dc", "C", "use_bias"):
        g[k] = int(g[k])
    g["score_type"] = str(g["score_type"])
    table = g["table"]
    g["E"] = table[g["his_ids"]]
    g["cand"] = table[g["cand_ids"]]
    g["metrics"] = {str(k): float(v) for k, v in zip(g["metric_names"], g["metric_values"])}
    return g


@pytest.fixture(params=golden_names())
def golden(request):
    return load_golden(request.param)


# MINER_TOL_REPORT=path: record every parity check (test, rtol, rms floor, worst fraction of the
# tolerance) so the bf16 bounds can be set from observed margins (tools/gpu_tol.sh)
if os.environ.get("MINER_TOL_REPORT"):
    import json

    from oracle import miner_oracle as _orc

    _orig_parity_ok = _orc.parity_ok

    def _recording_parity_ok(x, ref, *a, **kw):
        ok, worst = _orig_parity_ok(x, ref, *a, **kw)
        rec = {"test": os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0], "args": [float(v) for v in a],
               "kw": {k: float(v) for k, v in kw.items()}, "worst": float(worst), "ok": bool(ok)}
        with open(os.environ["MINER_TOL_REPORT"], "a") as f:
            f.write(json.dumps(rec) + "\n")
        return ok, worst

    _orc.parity_ok = _recording_parity_ok
