#!/bin/bash
# A/B of the compile-time MIND shape (L = 50, K = 32) against the run-time one (MINER_NEWS_SHP_RT),
# bf16 at d = 768 / 256 and fp32 at d = 256, then the news parity tests.
set -euo pipefail
O=gpurun_out/shp; mkdir -p $O
for DT in bf16 fp32; do for D in 768 256; do
  [ $DT = fp32 ] && [ $D = 768 ] && continue
  AB_D=$D AB_ALT=MINER_NEWS_SHP_RT timeout -k 10 200 python3 tools/news_ab.py $DT $([ $D = 768 ] && echo 1000000 || echo 400000) 9
done; done > $O/ab2.txt 2>&1
cat $O/ab2.txt
timeout -k 10 400 python3 -u -m pytest tests -m gpu -k "news or modules or fullsize or eval_loop or gather or parity" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
