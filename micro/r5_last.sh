#!/bin/bash
# final tree: full GPU suite, smoke, the driver's bench command
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r5_last_tests.txt 2>&1 || { tail -40 gpurun_out/r5_last_tests.txt; exit 1; }
tail -1 gpurun_out/r5_last_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_last_smoke.txt 2>&1 || { tail -20 gpurun_out/r5_last_smoke.txt; exit 1; }
tail -1 gpurun_out/r5_last_smoke.txt
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5_last_bench.json 2> gpurun_out/r5_last_bench.err || { tail -20 gpurun_out/r5_last_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r5_last_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['cpu_baseline']['value'], (d.get('steady_state') or {}).get('scans_per_s'), d.get('gpu_vs_cpu'))"
