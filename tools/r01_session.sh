#!/bin/bash
# Round-1 closing session (runs here, one gpurun call at a time): news-kernel parity + timing after
# the padding-DMA skip (reverted if its tests fail), the full GPU check, the news-path profiles.
set -u
cd /root/repo
S=gpurun_out/session.txt
G=/usr/local/graft/bin/gpurun
say() { echo "[session $(date +%H:%M:%S)] $*" >> "$S"; }
run() {   # run <out> <timeout> <command>; retried only when no box was free (exit 3)
  local rc
  for a in 1 2 3 4 5 6; do
    "$G" --timeout "$2" -- "$3" > "$1" 2>&1; rc=$?
    [ $rc -ne 3 ] && return $rc
    say "no box (try $a)"; sleep 120
  done
  return $rc
}
say start
run gpurun_out/skip1.out 900 'mkdir -p gpurun_out/skip1 && timeout -k 10 600 python3 -u -m pytest tests/test_gpu_news.py tests/test_gpu_eval_loop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/skip1/t.txt 2>&1 && timeout -k 10 120 python3 tools/news_time.py > gpurun_out/skip1/time.txt 2>&1 && timeout -k 10 120 python3 tools/news_time.py 4000 >> gpurun_out/skip1/time.txt 2>&1 && timeout -k 10 120 python3 tools/news_time.py 104000 32768 fp32 >> gpurun_out/skip1/time.txt 2>&1'
rc=$?; say "skip1 rc=$rc"
if [ $rc -ne 0 ]; then say revert; git checkout miner_amd/csrc/news.hip; python3 -m miner_amd.build >> "$S" 2>&1; fi
run gpurun_out/check2.out 1000 'bash tools/gpu_check.sh r01_check2'; say "check2 rc=$?"
run gpurun_out/prof5.out 900 'bash tools/news_profile.sh r01_news_v5'; say "prof5 rc=$?"
say done
