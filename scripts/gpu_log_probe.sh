# Write-log timing probes: shipped build over the whole pool and confined to
# 2 GiB (locality), plus ablation builds (timing only, wrong results).
set -u
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "partial or write_log or beyond" 2>&1 | tail -2 || exit 1
for args in "" "--span-gib 2" "--span-gib 0.5" "--delta"; do
  timeout -k 10 120 python -u scripts/prof_log.py --reps 8 $args || exit 1
done
for v in abl5 abl4; do
  echo "variant $v"; timeout -k 10 120 python -u scripts/prof_log.py --reps 8 --lib build/variants/libcurvecrc_$v.so || exit 1
done
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_log_c
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_log_c -o run --output-format csv -- python3 $R/scripts/prof_log.py > /dev/null 2>&1 || exit 1
echo done
