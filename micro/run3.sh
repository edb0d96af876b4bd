#!/bin/bash
# GPU suite, then (only when nothing faulted) the sort-site kernel probes
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/t4.log 2>&1
rc=$?
echo "pytest rc $rc"; tail -6 gpurun_out/t4.log
if [ $rc -gt 1 ] || grep -qai "illegal memory\|memory access fault\|hipErrorLaunchFailure\|core dumped" gpurun_out/t4.log; then echo "stop: fault or crash"; exit 3; fi
bash micro/sort_probe.sh && ALOAM_LIB_PATH=$PWD/micro/_var_pst/libaloam_hip.so timeout -k 10 200 python3 micro/ps_levels.py 2000 6000 25000 > gpurun_out/psl3.log 2>&1; cat gpurun_out/psl3.log | head -30
