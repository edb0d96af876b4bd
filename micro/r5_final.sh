#!/bin/bash
# round-5 final evidence: the driver's bench command (full line: roofline with the FETCH_SIZE pass, CPU baseline,
# C4 registration), its kernel trace at the same config, and the new s2m test
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_s2m.py -m gpu -x -q --timeout 200 --timeout-method thread -k "one_launch or invariance" > gpurun_out/r5_s2m_t2.txt 2>&1 || { tail -30 gpurun_out/r5_s2m_t2.txt; exit 1; }
tail -1 gpurun_out/r5_s2m_t2.txt
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5_bench_final.json 2> gpurun_out/r5_bench_final.err || { tail -20 gpurun_out/r5_bench_final.err; exit 1; }
tail -1 gpurun_out/r5_bench_final.json | cut -c1-1500
NAME=r5final STEPS=20 bash micro/r4_prof.sh || exit 1
f=$(find gpurun_out/r5final -name "*kernel_trace.csv" | head -1)
python micro/frames.py $f 6 24 > gpurun_out/r5final_frames.txt && python micro/frames.py $f 182 219 >> gpurun_out/r5final_frames.txt
head -20 gpurun_out/r5final_frames.txt
