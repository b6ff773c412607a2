# SQ instruction mix / wait cycles of range_crc_kernel (WAL replay) and
# read_verify_kernel (verify on read): one counter group per pass
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for drv in prof_wal prof_reads; do
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass -d $R/gpurun_out/pmc_w_${drv}_$i -o run --output-format csv -- python3 $R/scripts/$drv.py > $R/gpurun_out/pmc_w_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc_w_$i.log; exit 1; }
done
done
echo pmc done
