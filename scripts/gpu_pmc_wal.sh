# SQ instruction mix / wait cycles and HBM bytes of the range kernel (WAL replay)
# beside the page kernel's, the same counter groups over each driver: one
# counter group per pass, never with tracing.  usage: gpu_pmc_wal.sh TAG [drivers...]
# (drivers: prof_wal prof_page prof_reads; default prof_wal prof_page)
set -u
R=$(pwd)
TAG=${1:-r04}
shift || true
DRV=${*:-prof_wal prof_page}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for drv in $DRV; do
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum"; do
  i=$((i+1))
  a=""; [ $drv = prof_page ] && a="--n 2"
  timeout -s KILL 90 rocprofv3 --pmc $pass -d $R/gpurun_out/pmc_w_${TAG}_${drv}_$i -o run --output-format csv -- python3 $R/scripts/$drv.py $a > $R/gpurun_out/pmc_w_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc_w_${TAG}_$i.log; exit 1; }
done
done
echo pmc done
