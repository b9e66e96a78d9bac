set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04f
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5.py -x -v --timeout 300 --timeout-method thread -k "fbmc or stage_variants or c5_fbmc" > gpurun_out/r04f/pytest.log 2>&1 || { echo pytest_fail; tail -30 gpurun_out/r04f/pytest.log; exit 1; }
tail -2 gpurun_out/r04f/pytest.log
for c in c3 c4; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --config $c --steps 5 --warmup 1 > gpurun_out/r04f/bench_$c.log 2>&1 || { echo bench_fail; tail -5 gpurun_out/r04f/bench_$c.log; exit 1; }
  tail -1 gpurun_out/r04f/bench_$c.log | cut -c1-200
done
echo r04f_done
