#!/bin/bash
# PMC passes (one counter group per pass, never with tracing domains) over
# scripts/prof_page.py.  Output: gpurun_out/pmc_<tag>/<pass>/run_counter_collection.csv
set -u
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU"; do
    name=$(echo "$pass" | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $pass -d "$OUT/$name" -o run --output-format csv -- \
        python3 "$R/scripts/prof_page.py" --n 2 > "$OUT/$name.log" 2>&1 || { echo "pass $name failed rc=$?"; exit 1; }
done
echo "pmc done: $OUT"
