# Round 3, first box: the new exchange-agreement tests, a 2-rank gloo bench
# rehearsal with a failure injected on rank 1, then the driver's round-end order.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_distributed_gpu.py tests/test_geometries.py tests/test_integrity_gpu.py tests/test_host_cpp.py -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r03a_dist.log 2>&1 || { echo DISTFAIL; tail -40 $R/gpurun_out/r03a_dist.log; exit 1; }
tail -1 $R/gpurun_out/r03a_dist.log
BENCH_DIST_BACKEND=gloo CC_INJECT_COMM_INIT_FAIL_RANK=1 timeout -k 10 300 python bench.py --gpus 2 --chunks 64 --steps 5 --warmup 2 --comm-timeout-ms 5000 --stream-chunks-per-rank 32 > $R/gpurun_out/r03a_gloo2.log 2>&1 || { echo GLOOFAIL; tail -30 $R/gpurun_out/r03a_gloo2.log; exit 1; }
tail -1 $R/gpurun_out/r03a_gloo2.log
bash scripts/gpu_round_end_rehearsal.sh
