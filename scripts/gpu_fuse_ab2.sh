# Metapage chunks first in the page kernel's tail (fused2) vs last (fused) vs HEAD (base).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused or config1 or dynamic_tail or geometr" -m gpu -x -q --timeout 200 --timeout-method thread > $R/gpurun_out/fuse2_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/fuse2_tests.log; exit 1; }
tail -1 $R/gpurun_out/fuse2_tests.log
timeout -k 10 400 python -u scripts/pool_ab.py build/variants/libcurvecrc_base.so build/variants/libcurvecrc_fused2.so build/variants/libcurvecrc_fused.so > $R/gpurun_out/fuse2_pool_ab.log 2>&1 || { echo POOLABFAIL; tail -20 $R/gpurun_out/fuse2_pool_ab.log; exit 1; }
tail -4 $R/gpurun_out/fuse2_pool_ab.log
echo done
