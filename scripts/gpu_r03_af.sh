# HBM traffic of the secondary kernels (PMC, one counter group per pass):
# verify on read (scripts/prof_reads.py) and WAL replay (scripts/prof_wal.py).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
PMC_PASSES="FETCH_SIZE|WRITE_SIZE" PMC_DRIVER=scripts/prof_reads.py bash scripts/gpu_pmc_log.sh _r03_reads || exit 1
PMC_PASSES="FETCH_SIZE|WRITE_SIZE" PMC_DRIVER=scripts/prof_wal.py bash scripts/gpu_pmc_log.sh _r03_wal || exit 1
tail -2 $R/gpurun_out/pmc_log_FETCH_SIZE_r03_reads.log $R/gpurun_out/pmc_log_FETCH_SIZE_r03_wal.log
echo done
