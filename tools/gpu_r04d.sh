set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04d
timeout -k 10 420 python -u -m pytest tests/test_gpu_poly.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04d/pytest_poly.log 2>&1 || { echo pytest_poly_fail; tail -30 gpurun_out/r04d/pytest_poly.log; exit 1; }
tail -2 gpurun_out/r04d/pytest_poly.log
bash tools/gpu_prof_quick.sh c3poly3 c3 --option pic_poly=1 || exit 1
tail -1 gpurun_out/pq_c3poly3/stats.log | cut -c1-250
echo r04d_done
