#!/bin/bash
# fused filter diagnosis: cube workgroups of k_rb_filter2 only (segment sorts and sums as separate launches)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ALOAM_RB_FUSED_DBG=2 timeout -k 10 120 python -u -m pytest tests/test_gpu_mapping.py -m gpu -x -v --timeout 100 --timeout-method thread -k "publication_surface" > gpurun_out/r5_fdbg.txt 2>&1 || { grep "E  \|passed\|failed" gpurun_out/r5_fdbg.txt | head; exit 1; }
tail -1 gpurun_out/r5_fdbg.txt
