set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04e
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5.py -x -v --timeout 300 --timeout-method thread -k "fbmc or stage_variants or c5_fbmc" > gpurun_out/r04e/pytest.log 2>&1 || { echo pytest_fail; tail -30 gpurun_out/r04e/pytest.log; exit 1; }
tail -2 gpurun_out/r04e/pytest.log
for o in wrow=0 wrow=1; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --config c3 --steps 5 --warmup 1 --option $o > gpurun_out/r04e/bench_c3_$o.log 2>&1 || { echo bench_fail; tail -5 gpurun_out/r04e/bench_c3_$o.log; exit 1; }
  tail -1 gpurun_out/r04e/bench_c3_$o.log | cut -c1-200
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config c5 --steps 3 --warmup 1 > gpurun_out/r04e/bench_c5.log 2>&1 || { echo bench5_fail; tail -5 gpurun_out/r04e/bench_c5.log; exit 1; }
tail -1 gpurun_out/r04e/bench_c5.log | cut -c1-200
echo r04e_done
