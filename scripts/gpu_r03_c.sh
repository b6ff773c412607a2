# Round-3 evidence for the shipped kernels: kernel trace + stats of the bench,
# kernel traces of the write log alone (full and delta), and PMC passes over
# the write log (HBM bytes and the SQ mix, one counter group per pass).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
bash scripts/gpu_profile.sh r03c 20 || { echo PROFFAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
for mode in full delta; do
  extra=""; [ $mode = delta ] && extra="--delta"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_log_r03c_$mode -o run --output-format csv -- python3 $R/scripts/prof_log.py --reps 10 $extra > $R/gpurun_out/prof_log_r03c_$mode.log 2>&1 || { echo LOGTRACEFAIL; exit 1; }
done
cd $R
bash scripts/gpu_pmc_log.sh _r03c || exit 1
bash scripts/gpu_pmc_log.sh _r03c_delta --delta || exit 1
echo done
