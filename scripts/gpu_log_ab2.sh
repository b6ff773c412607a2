# write-log parity tests on the in-tree build, then interleaved in-process A/B
# (scripts/log_ab.py) of the in-tree build against build/variants/<v> for each v
set -u
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "partial or write_log or beyond or integrity" 2>&1 | tail -3 || exit 1
L="curve_amd/libcurvecrc.so"
for v in "$@"; do L="$L build/variants/libcurvecrc_$v.so"; done
timeout -k 10 200 python -u scripts/log_ab.py $L || exit 1
timeout -k 10 200 python -u scripts/log_ab.py --delta $L || exit 1
echo done
