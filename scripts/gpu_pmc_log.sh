# PMC pass over the write-log kernel (scripts/prof_log.py), counters in ONE pass
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $R/gpurun_out/pmc_log -o run --output-format csv -- python3 $R/scripts/prof_log.py --reps 2 > $R/gpurun_out/pmc_log.log 2>&1
echo "rc=$?"
