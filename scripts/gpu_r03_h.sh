# Write log: one-piece pages' edge geometry precomputed per lane at metadata
# time (geo) vs recomputed with scalar math in every step (geo0 = previous
# build).  Parity of the write-log tests (both modes) and the C++ host layer,
# then interleaved A/B, full mode (delta mode does not use this path).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_host_cpp.py -m gpu -x -q --timeout 200 --timeout-method thread -k "log or partial or write or host" > $R/gpurun_out/h_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/h_tests.log; exit 1; }
tail -1 $R/gpurun_out/h_tests.log
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_geo0.so $V/libcurvecrc_geo.so > $R/gpurun_out/h_ab_full.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/h_ab_full.log; exit 1; }
tail -2 $R/gpurun_out/h_ab_full.log
echo done
