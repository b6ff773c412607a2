# flat vs sorted range schedule: parity tests, then in-process A/B (args: variants)
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "crc_ranges or wal" > $R/gpurun_out/wal_flat_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/wal_flat_tests.log; exit 1; }
tail -1 $R/gpurun_out/wal_flat_tests.log
timeout -k 10 200 python -u scripts/wal_sched_ab.py "$@" 2>&1 | grep -v amdgpu.ids | tee $R/gpurun_out/wal_flat_ab.log
