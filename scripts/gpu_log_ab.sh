# write-log A/B: parity tests on the shipped build, then timings of the
# shipped build and of build/variants/libcurvecrc_<v>.so for each v given
set -u
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "partial or write_log or beyond or integrity" 2>&1 | tail -2 || exit 1
for rep in 1 2; do
  timeout -k 10 120 python -u scripts/prof_log.py --reps 8 || exit 1
  timeout -k 10 120 python -u scripts/prof_log.py --reps 8 --delta || exit 1
  for v in "$@"; do
    echo "variant $v"
    timeout -k 10 120 python -u scripts/prof_log.py --reps 8 --lib build/variants/libcurvecrc_$v.so || exit 1
    timeout -k 10 120 python -u scripts/prof_log.py --reps 8 --delta --lib build/variants/libcurvecrc_$v.so || exit 1
  done
done
echo done
