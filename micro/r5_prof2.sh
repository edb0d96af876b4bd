#!/bin/bash
# kernel trace of the default C3 bench (20 steps + the late window) -> per-frame mapping / front breakdown at the
# headline frames (6-23) and in the steady-state window (182-219)
set -o pipefail
mkdir -p gpurun_out
N=${NAME:-r5p}
bash profiles/prof.sh $N --steps 20 --warmup 5 --no-traffic --c4-launches 0 --c4-reg-steps 0 || { tail gpurun_out/$N.log; exit 1; }
f=$(find gpurun_out/$N -name "*kernel_trace.csv" | head -1)
python micro/frames.py $f 6 24 16 > gpurun_out/${N}_frames.txt
python micro/frames.py $f 182 219 16 >> gpurun_out/${N}_frames.txt
s=$(find gpurun_out/$N -name "*kernel_stats.csv" | head -1)
cp $s gpurun_out/${N}_kernel_stats.csv
rm -f $f
cat gpurun_out/${N}_frames.txt
