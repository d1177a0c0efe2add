"""Every PMC counter file the bench line binds (bench.py load_pmc) was taken on the kernel sources
as they are now: its source_sha16 (tools/srcsha.py: the bytes of the family's kernel source, shared
header and C-ABI header, plus per-file build flags) equals the current one. An edit to a kernel
after its counter pass makes the bench report traffic / busy as null; this test says so on CPU."""
import json
import os

import pytest

from tools.srcsha import KERNEL_SOURCES, source_sha16

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOUND = {
    "pmc_traffic_news_x2.json": "news_x2", "pmc_traffic_news_x2_loss.json": "news_x2",
    "pmc_traffic_news_x2_full.json": "news_x2", "pmc_traffic_news_c2_x2.json": "news_x2",
    "pmc_traffic_news.json": "news", "pmc_traffic_news_c2.json": "news", "pmc_traffic_news_fp32.json": "news",
    "pmc_traffic.json": "miner_score", "pmc_traffic_dense_fp32.json": "miner_score",
    "pmc_traffic_ff_bf16.json": "fastformer", "pmc_traffic_rk_fp16.json": "corpus",
}


@pytest.mark.parametrize("name,family", sorted(BOUND.items()))
def test_counter_file_matches_current_sources(name, family):
    with open(os.path.join(ROOT, "profiles", name)) as f:
        t = json.load(f)
    assert t["source_files"] == list(KERNEL_SOURCES[family])
    assert t["source_sha16"] == source_sha16(KERNEL_SOURCES[family]), \
        f"{name}: kernel sources changed after the counter pass (re-run tools/r06_pmc.sh)"
