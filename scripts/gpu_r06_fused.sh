#!/bin/bash
# round 6: the scan epilogue fused into the page kernel (measured, reverted: profiles/fused_epilogue_ab_r06.txt) -- parity tests, then the step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    "tests/test_gpu_parity.py::test_full_size_config1_scan_step" "tests/test_gpu_parity.py::test_pool_scan_fused_metapages_and_tail_reuse" \
    tests/test_pool_native.py ${FUSED_TESTS:-} > gpurun_out/fused_tests.txt 2>&1 || { tail -40 gpurun_out/fused_tests.txt; exit 1; }
tail -2 gpurun_out/fused_tests.txt
B="python -u bench.py --steps 20 --warmup 5 --updates 0 --reads 0 --wal-entries 0 --no-e2e --no-cpu-baseline --no-pmc"
for r in 1 2; do
  timeout -k 10 200 $B > gpurun_out/fused_on_$r.json 2>/dev/null || exit 1
  CC_AB_NO_FUSED_EPILOGUE=1 timeout -k 10 200 $B > gpurun_out/fused_off_$r.json 2>/dev/null || exit 1
done
for f in gpurun_out/fused_o*_?.json; do python -c "
import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);r=d['roofline']
print('$f', d['value'], d['ms_per_step'], r['kernel_ms_avg'], round(d['ms_per_step']-r['kernel_ms_avg'],4), d['digest_check_cpu']['ok'])"; done
