# Write log: row offsets in the instruction's offset field (103 / 120 VGPRs),
# delta mode at 16 waves, two-piece pages' list in one round trip.  Parity of
# the write-log tests (both modes) and the C++ host layer, then interleaved A/B
# full and delta against the previous build and the two single-change builds.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_host_cpp.py -m gpu -x -q --timeout 200 --timeout-method thread -k "log or partial or write or host" > $R/gpurun_out/e_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/e_tests.log; exit 1; }
tail -1 $R/gpurun_out/e_tests.log
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_cur.so $V/libcurvecrc_new.so $V/libcurvecrc_new2.so $V/libcurvecrc_nomf.so > $R/gpurun_out/e_ab_full.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/e_ab_full.log; exit 1; }
tail -4 $R/gpurun_out/e_ab_full.log
timeout -k 10 300 python -u scripts/log_ab.py --delta $V/libcurvecrc_cur.so $V/libcurvecrc_new.so $V/libcurvecrc_d12.so $V/libcurvecrc_nomf.so > $R/gpurun_out/e_ab_delta.log 2>&1 || { echo ABDFAIL; tail -20 $R/gpurun_out/e_ab_delta.log; exit 1; }
tail -4 $R/gpurun_out/e_ab_delta.log
echo done
