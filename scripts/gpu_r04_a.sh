# round 4: the new GPU tests (bounded exchange, pseudo streams, integrity format errors), then the quad A/B and profile
set -u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "comm_wait or pseudo_streams or rank_lost or product_geometry or racy" > gpurun_out/r04a_tests.log 2>&1
rc=$?; tail -12 gpurun_out/r04a_tests.log; [ $rc = 0 ] || exit 1
bash scripts/gpu_quad.sh old rowplain && bash scripts/gpu_quad_prof.sh
