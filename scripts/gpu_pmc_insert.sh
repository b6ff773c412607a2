# PMC passes over the write-log path (scripts/prof_log.py): instruction mix and
# wait cycles of log_insert_kernel / log_pages_kernel (one counter group per pass)
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass -d $R/gpurun_out/pmc_ins_$i -o run --output-format csv -- python3 $R/scripts/prof_log.py --reps 2 > $R/gpurun_out/pmc_ins_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc_ins_$i.log; exit 1; }
done
echo pmc done
