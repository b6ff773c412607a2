# Write log: a batch's page CRCs stored by one instruction after the batch (and
# in delta mode the stored CRCs loaded by one instruction at metadata time):
# cb, shipped as the in-tree build; cb0 = one store / load per page.  Parity
# of the write-log tests (both modes) and the host layer, then A/B full and delta.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_host_cpp.py tests/test_integrity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "log or partial or write or host or integrity" > $R/gpurun_out/t_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/t_tests.log; exit 1; }
tail -1 $R/gpurun_out/t_tests.log
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_cb0.so $V/libcurvecrc_cb.so > $R/gpurun_out/t_ab.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/t_ab.log; exit 1; }
tail -2 $R/gpurun_out/t_ab.log
timeout -k 10 300 python -u scripts/log_ab.py --delta $V/libcurvecrc_cb0.so $V/libcurvecrc_cb.so > $R/gpurun_out/t_abd.log 2>&1 || { echo ABDFAIL; tail -20 $R/gpurun_out/t_abd.log; exit 1; }
tail -2 $R/gpurun_out/t_abd.log
echo done
