# Round evidence, part 2: PMC traffic passes of the page kernel (one counter
# group per pass), then kernel traces of the write-log and WAL-replay calls.
set -u
R=$(pwd)
TAG=${1:-r02}
bash $R/scripts/gpu_pmc.sh $TAG || { echo PMCFAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
for w in log wal; do
  rm -rf $R/gpurun_out/prof_${w}_$TAG
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${w}_$TAG -o run --output-format csv -- python3 $R/scripts/prof_$w.py > $R/gpurun_out/prof_${w}_$TAG.log 2>&1 || { echo ${w}PROFFAIL; exit 1; }
  grep "ms per" $R/gpurun_out/prof_${w}_$TAG.log
done
echo done
