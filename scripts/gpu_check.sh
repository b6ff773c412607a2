# One GPU call: the -m gpu tests, the default bench line, and a 2-rank gloo
# rehearsal of the multi-GPU bench on the one-GPU box (ranks share cuda:0).
# Each GPU step has its own time limit; the first failure ends the script.
set -u
R=$(pwd)
TAG=${1:-r02}
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $R/gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/gpu_tests_$TAG.log
timeout -k 10 400 python -u bench.py > $R/gpurun_out/bench_$TAG.log 2>&1 || { echo BENCHFAIL; tail -30 $R/gpurun_out/bench_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/bench_$TAG.log > $R/gpurun_out/bench_$TAG.json
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --chunks 256 --steps 5 --warmup 3 --stream-chunks-per-rank 200 > $R/gpurun_out/bench2_$TAG.log 2>&1 || { echo BENCH2FAIL; tail -30 $R/gpurun_out/bench2_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/bench2_$TAG.log
echo done
