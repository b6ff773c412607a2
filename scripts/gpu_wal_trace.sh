# kernel trace of one prof_wal run (range ordering pre-pass + range kernel)
set -u
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_walord
timeout -k 10 150 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_walord -o run --output-format csv -- python3 $R/scripts/prof_wal.py "$@" > $R/gpurun_out/prof_walord.log 2>&1 || exit 1
grep "ms per" $R/gpurun_out/prof_walord.log
