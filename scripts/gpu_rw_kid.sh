# WAL replay AND verify on read A/B of several builds under rocprofv3 (kernel time by Kernel_Id),
# after the range / WAL / verify parity tests on the in-tree build.
# usage: bash scripts/gpu_rw_kid.sh TAG A.so B.so [C.so ...]
set -u
R=$(pwd)
TAG=$1; shift
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "range or wal or bufs or masked or verify or read" > $R/gpurun_out/rw_kid_tests_$TAG.log 2>&1
rc=$?; tail -1 $R/gpurun_out/rw_kid_tests_$TAG.log; [ $rc = 0 ] || { tail -30 $R/gpurun_out/rw_kid_tests_$TAG.log; exit 1; }
L=""; for x in "$@"; do L="$L $R/$x"; done
O=$R/gpurun_out/rw_kid_$TAG.txt
echo "## wal: $*" > $O
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kid_w
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/kid_w -o run --output-format csv -- python3 $R/scripts/wal_ab.py $L 2>/dev/null | grep -v "^W2026\|^E2026" >> $O || exit 1
python3 $R/scripts/kid_ab.py $R/gpurun_out/kid_w range_flat_kernel 150 >> $O
rm -rf $R/gpurun_out/kid_w
echo "## verify on read: $*" >> $O
rm -rf $R/gpurun_out/kid_r
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/kid_r -o run --output-format csv -- python3 $R/scripts/reads_ab.py $L 2>/dev/null | grep -v "^W2026\|^E2026" >> $O || exit 1
python3 $R/scripts/kid_ab.py $R/gpurun_out/kid_r read_verify_kernel 60 >> $O
rm -rf $R/gpurun_out/kid_r
cat $O
