set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "knn_device" > gpurun_out/r5_knn2.txt 2>&1 || { tail -30 gpurun_out/r5_knn2.txt; exit 1; }
tail -1 gpurun_out/r5_knn2.txt
for gs in 8 4 16; do ALOAM_KNN_GS2=$gs timeout -k 10 120 python bench.py --c4-only --c4-launches 50 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['c4']; print('GS2=$gs', c['kernel'], round(c['ms']*1e3,2), 'us', round(c['streamed']/(c['ms']*1e-3)/16.8e12,4))"; done
