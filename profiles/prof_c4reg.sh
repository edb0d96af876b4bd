#!/bin/bash
# usage: profiles/prof_c4reg.sh NAME -- kernel-trace profile of the C4 sharded registration section
set -e
R=$PWD; N=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$N -o run --output-format csv -- python3 $R/bench.py --c4-reg-only "$@" > $R/gpurun_out/$N.log 2>&1
