# Round 3: every -m gpu test, a 2-rank gloo rehearsal of the N>1 bench with a
# failure injected into rank 1's native comm init, the per-XCD tail-head A/B
# (standalone page kernel and the whole scan step), then the driver's bench line.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $R/gpurun_out/r03b_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/r03b_tests.log; exit 1; }
tail -1 $R/gpurun_out/r03b_tests.log
BENCH_DIST_BACKEND=gloo CC_INJECT_COMM_INIT_FAIL_RANK=1 timeout -k 10 300 python bench.py --gpus 2 --chunks 64 --steps 5 --warmup 2 --comm-timeout-ms 5000 --stream-chunks-per-rank 32 > $R/gpurun_out/r03b_gloo2.log 2>&1 || { echo GLOOFAIL; tail -30 $R/gpurun_out/r03b_gloo2.log; exit 1; }
tail -1 $R/gpurun_out/r03b_gloo2.log
timeout -k 10 300 python -u scripts/ab_bench.py build/variants/libcurvecrc_heads1.so build/variants/libcurvecrc_heads8.so --rounds 15 > $R/gpurun_out/r03b_ab_heads.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/r03b_ab_heads.log; exit 1; }
cat $R/gpurun_out/r03b_ab_heads.log
timeout -k 10 300 python -u scripts/pool_ab.py build/variants/libcurvecrc_heads1.so build/variants/libcurvecrc_heads8.so > $R/gpurun_out/r03b_pool_ab.log 2>&1 || { echo POOLABFAIL; tail -20 $R/gpurun_out/r03b_pool_ab.log; exit 1; }
tail -8 $R/gpurun_out/r03b_pool_ab.log
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/r03b_bench.log 2>&1 || { echo BENCHFAIL; tail -30 $R/gpurun_out/r03b_bench.log; exit 1; }
tail -1 $R/gpurun_out/r03b_bench.log > $R/gpurun_out/r03b_bench.json
echo done
