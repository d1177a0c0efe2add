#!/bin/bash
# A/B of the fp32 news kernel's VALU candidate tail (1ee102c) against 03ddba5, news parity tests, a short bench.
set -euo pipefail
O=gpurun_out/tail; mkdir -p $O
timeout -k 10 300 python3 tools/bisect_news.py --dtype fp32 --B 1000000 --reps 7 03ddba5 1ee102c 1ee102c 03ddba5 > $O/ab.txt 2>&1
cat $O/ab.txt
timeout -k 10 400 python3 -u -m pytest tests -m gpu -k "news or modules or fullsize or eval_loop or gather or parity" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; b=json.load(open('$O/bench.json')); print(b['value'], b['roofline']['kernel_ms'], b['with_host_tolist'])"
