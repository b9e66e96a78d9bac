set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04b
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "skip or guard or bench_kernels_trace or error_counts_match" > gpurun_out/r04b/pytest.log 2>&1 || { echo pytest_fail; tail -30 gpurun_out/r04b/pytest.log; exit 1; }
tail -3 gpurun_out/r04b/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --option pic_skip=0 > gpurun_out/r04b/bench_noskip.log 2>&1 || { echo bench0_fail; tail -5 gpurun_out/r04b/bench_noskip.log; exit 1; }
tail -1 gpurun_out/r04b/bench_noskip.log | cut -c1-300
bash tools/gpu_bench_evidence.sh r04b c2 k_mic_data k_mic_data
