# A/B of the in-tree library against build/variants/*.so on the WAL replay
# shape (scripts/prof_wal.py); each library run twice, interleaved.
set -u
for rep in 1 2; do
  for lib in curve_amd/libcurvecrc.so build/variants/libcurvecrc_*.so; do
    [ -f "$lib" ] || continue
    echo "$lib"
    timeout -k 10 120 python3 scripts/prof_wal.py --lib "$lib" | grep -o "median [0-9.]* GB/s [0-9.]* spot_ok [A-Za-z]*" || exit 1
  done
done
