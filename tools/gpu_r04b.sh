set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04b
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "skip or guard or bench_kernels_trace or error_counts_match" > gpurun_out/r04b/pytest.log 2>&1 || { echo pytest_fail; tail -30 gpurun_out/r04b/pytest.log; exit 1; }
tail -3 gpurun_out/r04b/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 50 --option pic_skip=0 --option mic_lr=0 > gpurun_out/r04b/bench_old.log 2>&1 || { echo bench0_fail; tail -5 gpurun_out/r04b/bench_old.log; exit 1; }
tail -1 gpurun_out/r04b/bench_old.log | cut -c1-300
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 50 --option mic_lr=0 > gpurun_out/r04b/bench_skip.log 2>&1 || { echo bench1_fail; tail -5 gpurun_out/r04b/bench_skip.log; exit 1; }
tail -1 gpurun_out/r04b/bench_skip.log | cut -c1-300
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 50 --option mic_net=3 > gpurun_out/r04b/bench_pnm.log 2>&1 || { echo bench2_fail; tail -5 gpurun_out/r04b/bench_pnm.log; exit 1; }
tail -1 gpurun_out/r04b/bench_pnm.log | cut -c1-300
bash tools/gpu_bench_evidence.sh r04b c2 k_mic_data k_mic_data
