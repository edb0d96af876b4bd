#!/bin/bash
# One parameterised GPU driver (replaces the per-round rN_*.sh one-offs).
# usage: micro/gpu.sh TAG STEP [STEP ...]   (run from the repo root, under gpurun)
#   tests:<pytest -k expr>   GPU tests matching the expression          -> gpurun_out/TAG_tests.txt
#   suite                    the whole -m gpu suite + smoke()           -> gpurun_out/TAG_suite.txt, TAG_smoke.txt
#   bench[:<bench args>]     bench.py (default: the driver's command)   -> gpurun_out/TAG_bench.json / .err
#   c4prof                   rocprofv3 kernel trace of the C4 search     -> gpurun_out/TAG_c4/
#   c4pmc                    PMC passes over the C4 search               -> gpurun_out/TAG_pmc*/
#   prof[:<bench args>]      rocprofv3 kernel trace of bench.py          -> gpurun_out/TAG_prof/
#   py:<script args>         python -u <script args>                     -> gpurun_out/TAG_py.txt
# Every step has its own time limit; the first failing step ends the call (no GPU step after a failure).
set -o pipefail
R=$PWD
TAG=$1; shift
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fail() { echo "FAILED: $1"; tail -40 "$2"; exit 1; }
for S in "$@"; do
    case "$S" in
    tests:*)
        K="${S#tests:}"
        timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$K" \
            > gpurun_out/${TAG}_tests.txt 2>&1 || fail "$S" gpurun_out/${TAG}_tests.txt
        tail -1 gpurun_out/${TAG}_tests.txt ;;
    suite)
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
            > gpurun_out/${TAG}_suite.txt 2>&1 || fail suite gpurun_out/${TAG}_suite.txt
        tail -1 gpurun_out/${TAG}_suite.txt
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 \
            || fail smoke gpurun_out/${TAG}_smoke.txt
        tail -1 gpurun_out/${TAG}_smoke.txt ;;
    bench*)
        A="${S#bench}"; A="${A#:}"; [ -z "$A" ] && A="--gpus 1 --steps 20 --warmup 5"
        timeout -k 10 600 python bench.py $A > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
            || fail "$S" gpurun_out/${TAG}_bench.err
        python - gpurun_out/${TAG}_bench.json <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print("value", d.get("value"), "ms", d.get("ms_per_step"), "frac", r.get("frac"), "us", r.get("avg_launch_us"),
      "traffic", r.get("traffic"), r.get("traffic_error"), "cpu", (d.get("cpu_baseline") or {}).get("value"),
      "steady", (d.get("steady_state") or {}).get("scans_per_s"), "x", d.get("gpu_vs_cpu"),
      "c4reg", (d.get("c4_registration") or {}).get("value"), (d.get("c4_registration") or {}).get("pose_rel_vs_oracle"))
tt = (d.get("config") or {}).get("tictoc_ms") or {}
print({k: v for k, v in tt.items() if v})
print("steady tictoc", (d.get("steady_state") or {}).get("tictoc_ms"))
EOF
        ;;
    c4prof)
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_c4 \
            -o run --output-format csv -- python3 $R/bench.py --c4-only --c4-launches 20 ) > gpurun_out/${TAG}_c4.log 2>&1 \
            || fail c4prof gpurun_out/${TAG}_c4.log
        tail -2 gpurun_out/${TAG}_c4.log ;;
    c4pmc)
        i=0
        for C in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
            i=$((i + 1))
            ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/${TAG}_pmc$i \
                -o run --output-format csv -- python3 $R/bench.py --c4-only --c4-launches 5 ) > gpurun_out/${TAG}_pmc$i.log 2>&1 \
                || fail "pmc $C" gpurun_out/${TAG}_pmc$i.log
        done
        echo "pmc done" ;;
    pmc:*)
        # pmc:<label>:<counters...> — one PMC pass over the C4 search (bench.py --c4-only)
        L="${S#pmc:}"; N="${L%%:*}"; C="${L#*:}"
        ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/${TAG}_pmc_$N \
            -o run --output-format csv -- python3 $R/bench.py --c4-only --c4-launches 5 ) > gpurun_out/${TAG}_pmc_$N.log 2>&1 \
            || fail "pmc $C" gpurun_out/${TAG}_pmc_$N.log
        python micro/pmc_sum.py gpurun_out/${TAG}_pmc_$N ;;
    prof*)
        A="${S#prof}"; A="${A#:}"; [ -z "$A" ] && A="--steps 20 --warmup 5 --no-traffic --c4-reg-steps 0"
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof \
            -o run --output-format csv -- python3 $R/bench.py --no-cpu $A ) > gpurun_out/${TAG}_prof.log 2>&1 \
            || fail prof gpurun_out/${TAG}_prof.log
        tail -1 gpurun_out/${TAG}_prof.log ;;
    tpy:*)
        # kernel trace of a python script: tpy:<script args>
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_tpy \
            -o run --output-format csv -- python3 $R/${S#tpy:} ) > gpurun_out/${TAG}_tpy.log 2>&1 || fail "$S" gpurun_out/${TAG}_tpy.log
        python profiles/stats.py $(find gpurun_out/${TAG}_tpy -name "*kernel_stats.csv" | head -1) 1 30 ;;
    py:*)
        timeout -k 10 600 python -u ${S#py:} > gpurun_out/${TAG}_py.txt 2>&1 || fail "$S" gpurun_out/${TAG}_py.txt
        tail -15 gpurun_out/${TAG}_py.txt ;;
    *) echo "unknown step $S"; exit 2 ;;
    esac
done
echo "all steps ok"
