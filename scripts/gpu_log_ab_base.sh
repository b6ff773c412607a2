# write-log parity tests on the in-tree build, then the in-process A/B of the
# in-tree build against build/variants/libcurvecrc_base.so (a copy of the previous build), full and delta mode
set -u
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "partial or write_log or beyond or integrity or delta" 2>&1 | tail -2 || exit 1
timeout -k 10 200 python -u scripts/log_ab.py build/variants/libcurvecrc_base.so curve_amd/libcurvecrc.so || exit 1
timeout -k 10 200 python -u scripts/log_ab.py --delta build/variants/libcurvecrc_base.so curve_amd/libcurvecrc.so || exit 1
echo done
