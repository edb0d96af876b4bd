#!/bin/bash
# round-3 final evidence: GPU suite, default bench line, 200-step steady-state line, kernel trace (each step
# time-limited, stop at the first failure)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3f_gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3f_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r3f_bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/r3f_bench.log | head -1
timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps 200 > gpurun_out/r3f_bench200.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/r3f_bench200.log | head -1
bash profiles/prof.sh prof_r3f --steps 30 --no-traffic || exit 1
