# round 4: single-launch range kernel vs the round-3 two-launch one (build/variants/libcurvecrc_r3wal.so):
# the path's parity tests, the interleaved A/B, then a kernel trace of each
set -u
bash scripts/gpu_ab.sh wal r3wal || exit 1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in new r3wal; do
  lib=curve_amd/libcurvecrc.so; [ $v = r3wal ] && lib=build/variants/libcurvecrc_r3wal.so
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_wal_$v -o run --output-format csv -- python3 $R/scripts/prof_wal.py --lib $lib > $R/gpurun_out/kt_wal_$v.log 2>&1 || { echo "wal trace $v failed"; exit 1; }
done
echo wal done
