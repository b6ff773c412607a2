#!/bin/bash
# round 6: the C3 stream leg with a distinct host data pool -- the default (1,024 distinct 16 MiB
# chunks = 16 GiB pinned) and every one of the 10,000 chunks distinct (156 GiB pinned), each alone
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
COMMON="--steps 2 --warmup 1 --chunks 64 --updates 0 --reads 0 --wal-entries 0 --file-chunks 0 --no-cpu-baseline --no-pmc"
for D in 1024 10000; do
  T0=$(date +%s)
  timeout -k 10 400 python -u bench.py $COMMON --stream-distinct $D > gpurun_out/stream_d$D.json 2> gpurun_out/stream_d$D.err || { tail -30 gpurun_out/stream_d$D.err; exit 1; }
  echo "distinct $D: whole bench run $(( $(date +%s) - T0 )) s"
  python3 -c "import json;d=json.loads(open('gpurun_out/stream_d$D.json').read().strip().splitlines()[-1]);print($D, json.dumps(d.get('stream')))"
done
