# static range kernel: balance probes (args: variant names)
set -u
for rep in 1 2; do
  for v in "$@"; do
    echo "== $v random"; timeout -k 10 120 python -u scripts/prof_wal.py --lib build/variants/libcurvecrc_$v.so || exit 1
  done
  echo "== static sorted"; timeout -k 10 120 python -u scripts/prof_wal.py --sorted --lib build/variants/libcurvecrc_static.so || exit 1
done
