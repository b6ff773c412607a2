set -u
R=$(pwd)
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kid_e
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kid_e -o run --output-format csv -- python3 $R/scripts/pool_ab.py $R/curve_amd/libcurvecrc.so $R/build/variants/libcurvecrc_epi_noatomic.so $R/build/variants/libcurvecrc_epi_nomulmod.so 2>/dev/null | grep -v "^W2026\|^E2026" > $R/gpurun_out/epi_ab.txt || exit 1
python3 $R/scripts/kid_ab.py $R/gpurun_out/kid_e epilogue_kernel 60 >> $R/gpurun_out/epi_ab.txt
rm -rf $R/gpurun_out/kid_e
cat $R/gpurun_out/epi_ab.txt
