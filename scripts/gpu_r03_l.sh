# Kernel traces of verify-on-read (scripts/prof_reads.py) and WAL replay
# (scripts/prof_wal.py) alone: what each call spends outside its main kernel.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/l_reads -o run --output-format csv -- python3 $R/scripts/prof_reads.py --reps 10 > $R/gpurun_out/l_reads.log 2>&1 || { echo READSFAIL; tail -5 $R/gpurun_out/l_reads.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/l_wal -o run --output-format csv -- python3 $R/scripts/prof_wal.py > $R/gpurun_out/l_wal.log 2>&1 || { echo WALFAIL; tail -5 $R/gpurun_out/l_wal.log; exit 1; }
cd $R
for d in l_reads l_wal; do f=$(find gpurun_out/$d -name '*kernel_trace.csv' | head -1); python3 scripts/trace_summary.py "$f" gpurun_out/${d}_summary.json > /dev/null; python3 - "$f" > gpurun_out/${d}_timeline.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
prev = None
for r in rows[-40:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
    print(f"{n:60s} dur {(e - s) / 1e3:8.1f} us  gap {((s - prev) / 1e3 if prev else 0):7.1f} us")
    prev = e
PY
done
tail -3 gpurun_out/l_reads.log gpurun_out/l_wal.log
echo done
