#!/bin/bash
# usage: profiles/pmc.sh NAME "COUNTERS" cmd... -- one rocprofv3 PMC pass (counters only, no traces)
set -e
R=$PWD; N=$1; CNT=$2; shift 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc $CNT -d $R/gpurun_out/$N -o run --output-format csv -- "$@" > $R/gpurun_out/$N.log 2>&1
