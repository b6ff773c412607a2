# interleaved full-mode write-log timings: shipped build vs variants (args), 4 rounds
set -u
for rep in 1 2 3 4; do
  echo "== cur"; timeout -k 10 120 python -u scripts/prof_log.py --reps 12 || exit 1
  for v in "$@"; do echo "== $v"; timeout -k 10 120 python -u scripts/prof_log.py --reps 12 --lib build/variants/libcurvecrc_$v.so || exit 1; done
done
