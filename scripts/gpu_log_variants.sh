# write-log correctness (GPU tests) + A/B of library variants (build/variants/libcurvecrc_*.so)
set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "beyond_4gib or partial or write_log or full_size or verify_reads" > gpurun_out/tv.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/tv.log; exit 1; }
tail -1 gpurun_out/tv.log
for lib in curve_amd/libcurvecrc.so build/variants/libcurvecrc_*.so; do
  [ -f "$lib" ] || continue
  echo "$lib"
  timeout -k 10 120 python3 scripts/prof_log.py --lib $lib --reps 8 2>&1 | grep "ms per" || exit 1
done
