#!/bin/bash
# segment-size / fit sweep of the PCL-order sorts (cube filter, stack filter): C3 pipeline scans/s per config;
# then the GPU suite with the small-segment kernels forced (each step time-limited, stop at the first failure)
mkdir -p gpurun_out
for cfg in "ALOAM_X=0" "ALOAM_CUBE_SEG=2048" "ALOAM_CUBE_SEG=1024" "ALOAM_CUBE_SEG=2048 ALOAM_CUBE_FIT=2048" \
           "ALOAM_CUBE_SEG=2048 ALOAM_VOX_SEG=2048" "ALOAM_CUBE_SEG=2048 ALOAM_VOX_SEG=2048 ALOAM_VOX_FIT=4096" \
           "ALOAM_CUBE_SEG=1024 ALOAM_CUBE_FIT=2048 ALOAM_VOX_SEG=1024 ALOAM_VOX_FIT=2048"; do
  env $cfg timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps 200 > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
  echo "$cfg $(grep -o '"value": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"filter time": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"map prepare time": [0-9.]*' gpurun_out/sw.log | head -1)"
done
ALOAM_CUBE_SEG=1024 ALOAM_VOX_SEG=1024 ALOAM_VOX_FIT=2048 ALOAM_CUBE_FIT=2048 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/sw_tests.log 2>&1; rc=$?
tail -3 gpurun_out/sw_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u micro/s2m_share.py > gpurun_out/s2m_share.log 2>&1; tail -1 gpurun_out/s2m_share.log
