#!/bin/bash
# A/B of two more compile-time specialisations: the fp32 news kernel's plain-scoring form (no bias,
# no mui output; MINER_NEWS_PLAIN_RT = the SHP 1 form) and the ranker's K = 64 (MINER_RK_K_RT).
set -euo pipefail
O=gpurun_out/spec; mkdir -p $O
AB_ALT=MINER_NEWS_PLAIN_RT timeout -k 10 200 python3 tools/news_ab.py fp32 1000000 9 > $O/ab.txt 2>&1
AB_ENV=MINER_RK_K_RT timeout -k 10 300 python3 tools/corpus_ab.py 2048 200000 5 >> $O/ab.txt 2>&1
grep -v amdgpu.ids $O/ab.txt
