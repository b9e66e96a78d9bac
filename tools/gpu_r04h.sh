set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04h
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "bench_kernels_trace or error_counts_match or stage_variants or guard" > gpurun_out/r04h/pytest.log 2>&1 || { echo pytest_fail; tail -30 gpurun_out/r04h/pytest.log; exit 1; }
tail -1 gpurun_out/r04h/pytest.log
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 50 > gpurun_out/r04h/b_$i.log 2>&1 || { echo bench_fail; tail -5 gpurun_out/r04h/b_$i.log; exit 1; }
  tail -1 gpurun_out/r04h/b_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
done
