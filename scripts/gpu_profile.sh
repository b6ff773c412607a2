#!/bin/bash
# rocprofv3 kernel trace + stats of bench.py (run via gpurun from the repo root).
# PMC counters are collected separately by scripts/gpu_pmc.sh (never combined).
set -u
TAG=${1:-r01}
STEPS=${2:-20}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps "$STEPS" --warmup 10 --no-cpu-baseline --no-e2e --no-pmc > "$OUT/trace_bench.log" 2>&1 || exit $?
echo "profile done: $OUT"
