# Round 5: WAL replay / verify-on-read tail-constant re-sweep, kernel time by Kernel_Id
# from one interleaved rocprofv3 kernel-trace run per path (scripts/kid_ab.py), builds in
# load order: shipped, then the variants.  Each step bounded.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
O=$R/gpurun_out/tail_resweep.txt
: > $O
cd /tmp && export TMPDIR=/tmp
W="$R/curve_amd/libcurvecrc.so"; for v in w_div16 w_div64 w_blk8 w_blk32; do W="$W $R/build/variants/libcurvecrc_$v.so"; done
V="$R/curve_amd/libcurvecrc.so"; for v in r_div8 r_div32 r_slot16 r_slot64; do V="$V $R/build/variants/libcurvecrc_$v.so"; done
rm -rf $R/gpurun_out/kid_w
echo "## wal: shipped (1/32, 16 blocks), w_div16, w_div64, w_blk8, w_blk32" >> $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kid_w -o run --output-format csv -- python3 $R/scripts/wal_ab.py $W 2>/dev/null | grep -v "^W2026\|^E2026" >> $O || exit 1
python3 $R/scripts/kid_ab.py $R/gpurun_out/kid_w range_flat_kernel 150 >> $O
rm -rf $R/gpurun_out/kid_w
rm -rf $R/gpurun_out/kid_r
echo "## verify on read: shipped (1/16, 32 slots), r_div8, r_div32, r_slot16, r_slot64" >> $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kid_r -o run --output-format csv -- python3 $R/scripts/reads_ab.py $V 2>/dev/null | grep -v "^W2026\|^E2026" >> $O || exit 1
python3 $R/scripts/kid_ab.py $R/gpurun_out/kid_r read_verify_kernel 60 >> $O
rm -rf $R/gpurun_out/kid_r
cat $O
