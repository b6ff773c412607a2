# PMC passes over the write-log path (scripts/prof_log.py): HBM bytes (FETCH_SIZE,
# WRITE_SIZE: one pass each) and the SQ instruction mix, each in its own pass
# usage: gpu_pmc_log.sh [SUFFIX [driver args...]]  (e.g. "delta --delta")
# PMC_DRIVER=scripts/prof_reads.py profiles the verify-on-read path instead
set -u
R=$(pwd)
SUF=${1:-}
shift || true
PASSES=${PMC_PASSES:-"FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
IFS='|' read -ra PL <<< "$PASSES"
for pass in "${PL[@]}"; do
  name=$(echo "$pass" | cut -d' ' -f1)$SUF
  timeout -s KILL 90 rocprofv3 --pmc $pass -d $R/gpurun_out/pmc_log_$name -o run --output-format csv -- python3 $R/${PMC_DRIVER:-scripts/prof_log.py} --reps 2 "$@" > $R/gpurun_out/pmc_log_$name.log 2>&1 || { echo "pass $name failed"; exit 1; }
done
echo pmc done
