# interleaved A/B of range-kernel library variants (args: variant names; "cur" = in-tree)
set -u
lib() { [ "$1" = cur ] && echo curve_amd/libcurvecrc.so || echo build/variants/libcurvecrc_$1.so; }
for rep in 1 2; do
  for v in "$@"; do
    echo "== $v random"; timeout -k 10 120 python -u scripts/prof_wal.py --lib $(lib $v) || exit 1
    echo "== $v fixed"; timeout -k 10 120 python -u scripts/prof_wal.py --fixed 66048 --lib $(lib $v) || exit 1
  done
done
