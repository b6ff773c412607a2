set -u
for rep in 1 2; do
  timeout -k 10 120 python -u scripts/prof_wal.py || exit 1
  for v in "$@"; do echo "variant $v"; timeout -k 10 120 python -u scripts/prof_wal.py --lib build/variants/libcurvecrc_$v.so || exit 1; done
done
