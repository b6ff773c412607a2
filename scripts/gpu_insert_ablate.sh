# kernel traces of the write-log call for the in-tree build and insert-ablation variants
set -u
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in cur "$@"; do
  L=""; [ $v != cur ] && L="--lib $R/build/variants/libcurvecrc_$v.so"
  rm -rf $R/gpurun_out/prof_ins_$v
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ins_$v -o run --output-format csv -- python3 $R/scripts/prof_log.py --reps 8 $L > $R/gpurun_out/prof_ins_$v.log 2>&1 || { echo FAIL $v; tail -20 $R/gpurun_out/prof_ins_$v.log; exit 1; }
  echo "== $v"; grep -h "insert\|fillBuffer\|log_pages" $R/gpurun_out/prof_ins_$v/run_kernel_stats.csv | cut -d, -f1-4
done
echo done
