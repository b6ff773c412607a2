# Round 3 full rehearsal of the current tree: every -m gpu test, smoke(), the
# 2-rank gloo rehearsal with rank 1's native comm init failing, and the
# driver's bench line.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $R/gpurun_out/r03d_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/r03d_tests.log; exit 1; }
tail -1 $R/gpurun_out/r03d_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $R/gpurun_out/r03d_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $R/gpurun_out/r03d_smoke.log; exit 1; }
tail -1 $R/gpurun_out/r03d_smoke.log
BENCH_DIST_BACKEND=gloo CC_INJECT_COMM_INIT_FAIL_RANK=1 timeout -k 10 300 python bench.py --gpus 2 --chunks 64 --steps 5 --warmup 2 --comm-timeout-ms 5000 --stream-chunks-per-rank 32 > $R/gpurun_out/r03d_gloo2.log 2>&1 || { echo GLOOFAIL; tail -30 $R/gpurun_out/r03d_gloo2.log; exit 1; }
tail -1 $R/gpurun_out/r03d_gloo2.log
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/r03d_bench.log 2>&1 || { echo BENCHFAIL; tail -30 $R/gpurun_out/r03d_bench.log; exit 1; }
tail -1 $R/gpurun_out/r03d_bench.log > $R/gpurun_out/r03d_bench.json
cat $R/gpurun_out/r03d_bench.json
echo done
