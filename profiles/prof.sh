#!/bin/bash
# usage: profiles/prof.sh NAME [bench args...] -- kernel-trace profile of bench.py into gpurun_out/NAME
set -e
R=$PWD; N=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$N -o run --output-format csv -- python3 $R/bench.py --no-cpu "$@" > $R/gpurun_out/$N.log 2>&1
