# write-log kernel: unaligned vs 4-byte-aligned logs, kernel trace of each
set -u
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for al in 1 4; do
  rm -rf $R/gpurun_out/prof_log_a$al
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_log_a$al -o run --output-format csv -- python3 $R/scripts/prof_log.py --align $al > $R/gpurun_out/prof_log_a$al.log 2>&1 || exit 1
  grep "ms per" $R/gpurun_out/prof_log_a$al.log
done
