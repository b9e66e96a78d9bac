set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04c
timeout -k 10 420 python -u -m pytest tests/test_gpu_poly.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04c/pytest_poly.log 2>&1 || { echo pytest_poly_fail; tail -30 gpurun_out/r04c/pytest_poly.log; exit 1; }
tail -2 gpurun_out/r04c/pytest_poly.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 50 > gpurun_out/r04c/bench_c2.log 2>&1 || { echo bench_fail; tail -5 gpurun_out/r04c/bench_c2.log; exit 1; }
tail -1 gpurun_out/r04c/bench_c2.log | cut -c1-250
timeout -k 10 240 python -u bench.py --no-cpu-baseline --config c3 --steps 5 --warmup 1 --option pic_poly=1 > gpurun_out/r04c/bench_c3_poly.log 2>&1 || { echo benchc3p_fail; tail -5 gpurun_out/r04c/bench_c3_poly.log; exit 1; }
tail -1 gpurun_out/r04c/bench_c3_poly.log | cut -c1-250
bash tools/gpu_prof_quick.sh c3poly2 c3 --option pic_poly=1 || exit 1
echo r04c_done
