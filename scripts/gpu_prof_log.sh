# write log: rocprofv3 kernel trace + stats of the call, then PMC passes (SQ mix,
# HBM bytes, LDS/VMEM detail).  usage: gpu_prof_log.sh SUFFIX [prof_log.py args, e.g. --lib X.so]
set -u
R=$(pwd)
SUF=${1:-_log}
shift || true
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_log$SUF -o run --output-format csv -- python3 $R/scripts/prof_log.py --reps 4 "$@" > $R/gpurun_out/kt_log$SUF.log 2>&1 || { echo trace failed; exit 1; }
cd $R
PMC_PASSES="FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY|SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH" bash scripts/gpu_pmc_log.sh $SUF "$@" || exit 1
echo prof done
