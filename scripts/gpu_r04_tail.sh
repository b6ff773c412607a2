# round 4: the page kernel's tail counters zeroed one launch ahead (alternating
# slot sets) vs the round-3 arrival-counter reset (build/variants/libcurvecrc_r4pre.so):
# parity tests of the page / pool path, the page-kernel and scan-step A/B, then a
# translation / latency PMC pass over the page kernel and the WAL kernel
set -u
bash scripts/gpu_ab.sh page r4pre || exit 1
timeout -k 10 300 python -u scripts/pool_ab.py curve_amd/libcurvecrc.so build/variants/libcurvecrc_r4pre.so || exit 1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for drv in prof_page prof_wal; do
  a=""; [ $drv = prof_page ] && a="--n 2"
  timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum -d $R/gpurun_out/pmc_tlb_$drv -o run --output-format csv -- python3 $R/scripts/$drv.py $a > $R/gpurun_out/pmc_tlb_$drv.log 2>&1 || { echo "tlb pass $drv failed"; tail -5 $R/gpurun_out/pmc_tlb_$drv.log; exit 1; }
done
echo tail done
