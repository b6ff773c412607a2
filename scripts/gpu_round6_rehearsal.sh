# Round-6 evidence in one GPU call, in the driver's order: every -m gpu test, smoke(), the
# bench with the driver's flags (its own live PMC traffic passes inside), then the same bench
# command under rocprofv3 --kernel-trace --stats (no PMC: counters never ride with tracing; no host
# legs: their page-kernel launches over staging batches would share the 16 GiB launches' stats row).
# Each GPU step bounded; the first failure ends the call.  usage: bash scripts/gpu_round6_rehearsal.sh TAG
set -u
R=$(pwd)
TAG=${1:-r06}
mkdir -p $R/gpurun_out
if [ "${2:-}" != profile-only ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread > $R/gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/gpu_tests_$TAG.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" || { echo SMOKEFAIL; exit 1; }
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/bench_$TAG.log 2>&1 || { echo BENCHFAIL; tail -30 $R/gpurun_out/bench_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/bench_$TAG.log > $R/gpurun_out/bench_$TAG.json
fi
OUT=$R/gpurun_out/prof_$TAG
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-e2e --no-cpu-baseline > $OUT/trace_bench.log 2>&1 || { echo PROFFAIL; tail -20 $OUT/trace_bench.log; exit 1; }
S=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
cp "$S" $R/gpurun_out/rocprof_kernel_stats_$TAG.csv
python3 $R/scripts/trace_summary.py "$T" $R/gpurun_out/rocprof_bench_summary_$TAG.json > /dev/null
grep "^{" $OUT/trace_bench.log > $R/gpurun_out/bench_under_rocprof_$TAG.json
rm -rf $OUT/trace
echo done
