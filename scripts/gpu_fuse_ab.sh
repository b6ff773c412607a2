# Fused metapages + self-resetting tail counters, and the engine-owned write-log
# table the page kernel leaves clear: parity (pool scan, page-kernel tails,
# geometries, write log incl. the C++ host layer), then interleaved A/B of the
# scan step, the standalone page kernel and the write log against HEAD's build.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_geometries.py tests/test_pool_native.py tests/test_host_cpp.py -m gpu -x -q --timeout 200 --timeout-method thread > $R/gpurun_out/fuse_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/fuse_tests.log; exit 1; }
tail -1 $R/gpurun_out/fuse_tests.log
timeout -k 10 300 python -u scripts/pool_ab.py build/variants/libcurvecrc_base.so build/variants/libcurvecrc_fused.so > $R/gpurun_out/fuse_pool_ab.log 2>&1 || { echo POOLABFAIL; tail -20 $R/gpurun_out/fuse_pool_ab.log; exit 1; }
tail -3 $R/gpurun_out/fuse_pool_ab.log
timeout -k 10 300 python -u scripts/ab_bench.py build/variants/libcurvecrc_base.so build/variants/libcurvecrc_fused.so --rounds 15 > $R/gpurun_out/fuse_ab_page.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/fuse_ab_page.log; exit 1; }
tail -3 $R/gpurun_out/fuse_ab_page.log
timeout -k 10 300 python -u scripts/log_ab.py build/variants/libcurvecrc_base.so build/variants/libcurvecrc_logtab.so > $R/gpurun_out/logtab_ab.log 2>&1 || { echo LOGABFAIL; tail -20 $R/gpurun_out/logtab_ab.log; exit 1; }
tail -4 $R/gpurun_out/logtab_ab.log
timeout -k 10 300 python -u scripts/log_ab.py --delta build/variants/libcurvecrc_base.so build/variants/libcurvecrc_logtab.so > $R/gpurun_out/logtab_ab_delta.log 2>&1 || { echo LOGABDFAIL; tail -20 $R/gpurun_out/logtab_ab_delta.log; exit 1; }
tail -4 $R/gpurun_out/logtab_ab_delta.log
echo done
