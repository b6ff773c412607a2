# Write log: dynamic tail v2 (per-XCD counters, a drained counter skipped
# without an atomic) after the age-weighted static shares, vs none (t0); em = t0 + the first batch's head slots and table entries loaded during the LDS fill.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_host_cpp.py -m gpu -x -q --timeout 200 --timeout-method thread -k "log or partial or write or host" > $R/gpurun_out/r_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/r_tests.log; exit 1; }
tail -1 $R/gpurun_out/r_tests.log
V=build/variants
timeout -k 10 400 python -u scripts/log_ab.py $V/libcurvecrc_t0.so $V/libcurvecrc_t16k8.so $V/libcurvecrc_t32k4.so $V/libcurvecrc_t16k16.so $V/libcurvecrc_em.so > $R/gpurun_out/r_ab.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/r_ab.log; exit 1; }
tail -5 $R/gpurun_out/r_ab.log
echo done
