#!/bin/bash
# kernel-trace summary of the C3 pipeline at STEPS steps -> gpurun_out/NAME/*kernel_stats.csv
set -o pipefail
N=${NAME:-r4p}; ST=${STEPS:-200}
bash profiles/prof.sh $N --steps $ST --no-traffic --c4-launches 0 --c4-reg-steps 0 || exit 1
f=$(find gpurun_out/$N -name "*kernel_stats.csv" | head -1)
python profiles/stats.py $f $((ST + 13)) 25 > gpurun_out/$N.txt
