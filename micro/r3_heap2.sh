#!/bin/bash
# heap-job scheduling variants (hybrid default / lanes only / waves only): bench at 50 / 200 steps; then the
# GPU suite on the default build (each step time-limited, stop at the first failure)
mkdir -p gpurun_out
for st in 50 200; do
for lib in "" micro/_var_hl0/libaloam_hip.so micro/_var_hlinf/libaloam_hip.so; do
  ALOAM_LIB_PATH=$lib timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps $st > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
  echo "steps $st lib=$lib $(grep -o '"value": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"filter time": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"seperate points time": [0-9.]*' gpurun_out/sw.log | head -1)"
done; done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3h_gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3h_gpu_tests.log
exit $rc
