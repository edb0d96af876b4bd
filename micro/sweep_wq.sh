#!/bin/bash
# ls_sort wave-queue tail variants (micro/build_variant.sh builds): C3 pipeline scans/s at 50 and 200 steps
mkdir -p gpurun_out
for st in 50 200; do
for lib in "" micro/_var_wq256/libaloam_hip.so micro/_var_wq1024/libaloam_hip.so micro/_var_wq4096/libaloam_hip.so; do
  ALOAM_LIB_PATH=$lib timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps $st > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
  echo "steps $st lib=$lib $(grep -o '"value": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"filter time": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"map prepare time": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"seperate points time": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"ate_delta_vs_pcl_order_m": [0-9.e-]*' gpurun_out/sw.log | head -1)"
done; done
