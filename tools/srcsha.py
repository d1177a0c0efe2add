"""The source identity a PMC counter file is bound to (tools/pmc_traffic.py writes it, bench.py checks
it): sha256 over the repo-relative path and bytes of each kernel source a counter pass measured (and
its per-file build flags), so a kernel edited after its profiling pass cannot carry stale counters
into a bench line."""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# the sources each profiled kernel family is compiled from
KERNEL_SOURCES = {
    "news_x2": ("miner_amd/csrc/news_x2.hip", "miner_amd/csrc/cdna4_common.h", "include/miner_news.h"),
    "news": ("miner_amd/csrc/news.hip", "miner_amd/csrc/cdna4_common.h", "include/miner_news.h"),
    "miner_score": ("miner_amd/csrc/miner_score.hip", "miner_amd/csrc/cdna4_common.h", "include/miner_score.h"),
    "fastformer": ("miner_amd/csrc/fastformer.hip", "miner_amd/csrc/cdna4_common.h", "include/miner_fastformer.h"),
    "corpus": ("miner_amd/csrc/corpus.hip", "miner_amd/csrc/cdna4_common.h", "include/miner_corpus.h"),
}


def _file_flags(rel: str) -> list:
    """Extra hipcc flags miner_amd/build.py compiles this source with (they change the code as much
    as an edit does)."""
    import sys
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from miner_amd.build import FILE_FLAGS
    return FILE_FLAGS.get(os.path.basename(rel), [])


def source_sha16(files) -> str:
    h = hashlib.sha256()
    for rel in files:
        h.update(rel.encode())
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(f.read())
        fl = _file_flags(rel)
        if fl:
            h.update(repr(fl).encode())
    return h.hexdigest()[:16]
