#!/bin/bash
# larger segments / whole-cube LDS sorts: C3 pipeline scans/s at 50 and 200 steps per config
mkdir -p gpurun_out
for st in 50 200; do
for cfg in "ALOAM_X=0" "ALOAM_CUBE_SEG=8192" "ALOAM_CUBE_SEG=10240 ALOAM_CUBE_FIT=10240" "ALOAM_CUBE_SEG=8192 ALOAM_CUBE_FIT=10240 ALOAM_VOX_SEG=8192" \
           "ALOAM_CUBE_SEG=10240 ALOAM_CUBE_FIT=10240 ALOAM_VOX_SEG=10240"; do
  env $cfg timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps $st > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
  echo "steps $st $cfg $(grep -o '"value": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"filter time": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"map prepare time": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"scan registration time": [0-9.]*' gpurun_out/sw.log | head -1)"
done; done
