# Verify-on-read (cc_verify_reads_dev) A/B of several builds under rocprofv3: kernel time by
# Kernel_Id (load order), after the verify/read parity tests on the in-tree build.
# usage: bash scripts/gpu_reads_kid.sh TAG A.so B.so [C.so ...]
set -u
R=$(pwd)
TAG=$1; shift
L=""; for x in "$@"; do L="$L $R/$x"; done
mkdir -p $R/gpurun_out
O=$R/gpurun_out/reads_kid_$TAG.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "verify or read or masked" > $R/gpurun_out/reads_kid_tests_$TAG.log 2>&1
rc=$?; tail -1 $R/gpurun_out/reads_kid_tests_$TAG.log; [ $rc = 0 ] || exit 1
echo "## verify on read: $*" > $O
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kid_r
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/kid_r -o run --output-format csv -- python3 $R/scripts/reads_ab.py $L 2>/dev/null | grep -v "^W2026\|^E2026" >> $O || exit 1
python3 $R/scripts/kid_ab.py $R/gpurun_out/kid_r read_verify_kernel 60 >> $O
rm -rf $R/gpurun_out/kid_r
cat $O
