#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root):
#   1. rocprofv3 kernel trace + stats of bench.py (per-kernel durations)
#   2. separate PMC passes for FETCH_SIZE and WRITE_SIZE (never combined with
#      tracing domains), shorter run.
# Outputs under gpurun_out/prof_<tag>/ ; summaries are copied into profiles/ by hand.
set -u
TAG=${1:-r01}
STEPS=${2:-20}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps "$STEPS" --warmup 3 --no-cpu-baseline --no-e2e > "$OUT/trace_bench.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/pmc_write.log" 2>&1 || exit $?
echo "profile done: $OUT"
