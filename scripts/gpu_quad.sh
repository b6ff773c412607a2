# write-log quad kernel: parity tests of the write log, then an interleaved A/B
# of the shipped build against build/variants/libcurvecrc_<v>.so for each v given
set -u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "write_log or partial" > gpurun_out/quad_tests.log 2>&1
rc=$?; tail -5 gpurun_out/quad_tests.log; [ $rc = 0 ] || exit 1
libs=""
for v in "$@"; do libs="$libs build/variants/libcurvecrc_$v.so"; done
timeout -k 10 300 python -u scripts/log_ab.py curve_amd/libcurvecrc.so $libs || exit 1
timeout -k 10 300 python -u scripts/log_ab.py --delta curve_amd/libcurvecrc.so $libs || exit 1
echo done
