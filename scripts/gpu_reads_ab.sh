# verify-on-read: parity tests on the shipped build, then interleaved timings vs variants (args)
set -u
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "verify or read" 2>&1 | tail -2 || exit 1
for rep in 1 2 3; do
  echo "== cur"; timeout -k 10 120 python -u scripts/prof_reads.py || exit 1
  for v in "$@"; do echo "== $v"; timeout -k 10 120 python -u scripts/prof_reads.py --lib build/variants/libcurvecrc_$v.so || exit 1; done
done
