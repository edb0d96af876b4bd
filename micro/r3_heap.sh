#!/bin/bash
# wave heap sort: GPU suite, bench at 50 / 200 steps, kernel trace (each step time-limited, stop at the first failure)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3h_gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3h_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
for st in 50 200; do
  timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps $st > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
  echo "steps $st $(grep -o '"value": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"filter time": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"seperate points time": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"ate_delta_vs_pcl_order_m": [0-9.e-]*' gpurun_out/sw.log | head -1)"
done
bash profiles/prof.sh prof_r3h_200 --steps 200 --no-traffic --c4-launches 0 --c4-reg-steps 0 || exit 1
