#!/bin/bash
# round-3 final tree: GPU suite + default bench line (each step time-limited, stop at the first failure)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3f_gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3f_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r3f_bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/r3f_bench.log | head -1
