set -e
mkdir -p gpurun_out/gelu
timeout -k 10 300 python3 tools/bisect_news.py --dtype fp32 --B 1000000 --reps 7 b281ad5 03ddba5 03ddba5 b281ad5 > gpurun_out/gelu/ab.txt 2>&1
cat gpurun_out/gelu/ab.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "news or modules or fullsize or eval_loop" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gelu/tests.log 2>&1
tail -3 gpurun_out/gelu/tests.log
