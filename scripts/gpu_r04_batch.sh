# round 4: the pending A/Bs in one call (WAL pieces/tail, verify tail, write log G pages a wave)
set -u
bash scripts/gpu_r04_rr1.sh || exit 1
bash scripts/gpu_r04_group.sh || exit 1
