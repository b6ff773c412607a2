# What the driver runs at round end, in its order: every -m gpu test, smoke(),
# then the bench with the driver's flags.  Each step bounded; the first failure ends it.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $R/gpurun_out/gpu_tests_end.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/gpu_tests_end.log; exit 1; }
tail -1 $R/gpurun_out/gpu_tests_end.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" || { echo SMOKEFAIL; exit 1; }
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/bench_end.log 2>&1 || { echo BENCHFAIL; tail -30 $R/gpurun_out/bench_end.log; exit 1; }
tail -1 $R/gpurun_out/bench_end.log > $R/gpurun_out/bench_end.json
echo done
