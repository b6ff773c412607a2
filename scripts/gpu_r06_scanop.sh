#!/bin/bash
# round 6: the scan-op call shape (row f1) -- GPU tests, then the bench's scan_op leg alone
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_scan_op.py -m gpu \
    > gpurun_out/scanop_tests.txt 2>&1 || { tail -30 gpurun_out/scanop_tests.txt; exit 1; }
tail -3 gpurun_out/scanop_tests.txt
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --chunks 64 --updates 0 --reads 0 --wal-entries 0 \
    --stream-chunks 0 --file-chunks 0 --no-cpu-baseline --no-pmc ${BENCH_EXTRA:-} \
    > gpurun_out/scanop_bench.json 2> gpurun_out/scanop_bench.err || { tail -20 gpurun_out/scanop_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/scanop_bench.json').read().strip().splitlines()[-1]);print(json.dumps(d.get('scan_op'),indent=1));print('e2e',d.get('e2e_pinned_GiBps'))"
