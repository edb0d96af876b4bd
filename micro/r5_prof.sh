#!/bin/bash
# round-5 evidence pass: knn GPU tests, C4 search kernel trace + PMC passes (default kernel), C3 kernel trace at the
# driver's 20-step config (timeline), heap micro-benchmark. Every GPU step under its own time limit, chained with &&.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "knn_device" \
  > gpurun_out/r5_knn_tests.txt 2>&1 || { tail -30 gpurun_out/r5_knn_tests.txt; exit 1; }
tail -3 gpurun_out/r5_knn_tests.txt
bash profiles/prof.sh r5_c4 --c4-only --c4-launches 20 || { tail gpurun_out/r5_c4.log; exit 1; }
for p in "a FETCH_SIZE" "b TCC_HIT_sum TCC_MISS_sum" "c SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
  set -- $p; n=$1; shift
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc "$@" -d $R/gpurun_out/r5_pmc_$n -o run --output-format csv -- \
     python3 $R/bench.py --c4-only --c4-launches 5 > $R/gpurun_out/r5_pmc_$n.log 2>&1) || { tail $R/gpurun_out/r5_pmc_$n.log; exit 1; }
done
NAME=r5p20 STEPS=20 bash micro/r4_prof.sh || exit 1
f=$(find gpurun_out/r5p20 -name "*kernel_trace.csv" | head -1)
python micro/timeline.py $f 12 > gpurun_out/r5p20_timeline.txt
python micro/per_round.py $f k_map_assoc k_lm_coop > gpurun_out/r5p20_rounds.txt

timeout -k 10 120 python micro/heap_bench.py 64 300 1000 3000 > gpurun_out/r5_heap.txt 2>&1
cat gpurun_out/r5_heap.txt gpurun_out/r5p20_timeline.txt
