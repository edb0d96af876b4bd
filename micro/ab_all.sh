#!/bin/bash
# rebuild A/B (profiling aid): k_rb_cubevox phase probe, map/trajectory bit-identity of the fused rebuild
# vs ALOAM_REBUILD_FUSED=0 over N scans, then the mapping phase times in a pipeline bench run
N=${1:-60}
mkdir -p gpurun_out
timeout -k 10 200 python micro/rb_probe.py $N 2>&1 | grep -v amdgpu | sort -k3 -n -r | head -4
timeout -k 10 120 python micro/rebuild_ab.py $N gpurun_out/ab_fused.npz > gpurun_out/ab1.log 2>&1 || exit 1
ALOAM_REBUILD_FUSED=0 timeout -k 10 120 python micro/rebuild_ab.py $N gpurun_out/ab_old.npz > gpurun_out/ab0.log 2>&1 || exit 1
python - <<'PY' || exit 1
import numpy as np, sys
a = np.load("gpurun_out/ab_fused.npz"); b = np.load("gpurun_out/ab_old.npz")
bad = 0
for k in a.files:
    same = a[k].shape == b[k].shape and np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8))
    bad += not same
    print(k, a[k].shape, b[k].shape, "bit-identical" if same else "DIFFER")
sys.exit(bad)
PY
[ -n "$NOBENCH" ] && exit 0
ALOAM_MAP_PHASES=1 timeout -k 10 150 python bench.py --no-cpu --c4-launches 0 --c4-reg-steps 0 --steps 450 > gpurun_out/ph.log 2> gpurun_out/ph.err || exit 1
grep -a "map phases" gpurun_out/ph.err | tail -1
python -c "import json;d=json.loads(open('gpurun_out/ph.log').read().strip().splitlines()[-1]);print('bench',d['value'],d['ms_per_step'])"
