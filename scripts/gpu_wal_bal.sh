set -u
for rep in 1 2; do
  timeout -k 10 120 python -u scripts/prof_wal.py || exit 1
  timeout -k 10 120 python -u scripts/prof_wal.py --fixed 66048 || exit 1
  timeout -k 10 120 python -u scripts/prof_wal.py --sorted || exit 1
done
