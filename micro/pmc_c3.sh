#!/bin/bash
# two PMC passes over a short serial bench (per-kernel instruction / wait counters)
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $R/gpurun_out/pmcA -o run --output-format csv -- python3 $R/bench.py --mode serial --steps 10 --no-cpu --c4-launches 0 --c4-reg-steps 0 --no-traffic > $R/gpurun_out/pmcA.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_FLAT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM -d $R/gpurun_out/pmcB -o run --output-format csv -- python3 $R/bench.py --mode serial --steps 10 --no-cpu --c4-launches 0 --c4-reg-steps 0 --no-traffic > $R/gpurun_out/pmcB.log 2>&1
