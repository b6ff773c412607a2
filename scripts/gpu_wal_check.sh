set -u
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "range or wal or bufs or chunk_hash or golden or beyond" 2>&1 | tail -2 || exit 1
for rep in 1 2; do
  timeout -k 10 120 python -u scripts/prof_wal.py || exit 1
  timeout -k 10 120 python -u scripts/prof_wal.py --fixed 66048 || exit 1
  for v in "$@"; do echo "variant $v"; timeout -k 10 120 python -u scripts/prof_wal.py --lib build/variants/libcurvecrc_$v.so || exit 1; done
done
