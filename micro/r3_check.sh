#!/bin/bash
# round-3 check on the box: GPU suite, bench line, kernel-trace profile (each step time-limited, stop at the first failure)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r3_bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/r3_bench.log | head -1
bash profiles/prof.sh prof_r3 --steps 30 --no-traffic || exit 1
python profiles/stats.py gpurun_out/prof_r3 > gpurun_out/prof_r3_stats.txt 2>&1 || true
