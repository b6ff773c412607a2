mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pool_native.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --updates 0 > gpurun_out/b2.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/b2.log; exit 1; }
tail -1 gpurun_out/b2.log
BENCH_DIST_BACKEND=gloo timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --chunks 64 > gpurun_out/b2r.log 2>&1; echo "rehearsal rc=$?"
tail -3 gpurun_out/b2r.log
