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
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 50 > gpurun_out/r04b/bench_new.log 2>&1 || { echo bench3_fail; tail -5 gpurun_out/r04b/bench_new.log; exit 1; }
tail -1 gpurun_out/r04b/bench_new.log | cut -c1-300
# polyphase perfect-CSI passes (option pic_poly, off by default): parity, then C3 A/B.
# An assertion failure (rc 1) still lets the A/B run; anything else ends the call.
timeout -k 10 420 python -u -m pytest tests/test_gpu_poly.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04b/pytest_poly.log 2>&1
rc=$?
tail -3 gpurun_out/r04b/pytest_poly.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo pytest_poly_rc $rc; tail -30 gpurun_out/r04b/pytest_poly.log; exit 1; fi
timeout -k 10 240 python -u bench.py --no-cpu-baseline --config c3 --steps 5 --warmup 1 > gpurun_out/r04b/bench_c3_band.log 2>&1 || { echo benchc3_fail; tail -5 gpurun_out/r04b/bench_c3_band.log; exit 1; }
tail -1 gpurun_out/r04b/bench_c3_band.log | cut -c1-300
timeout -k 10 240 python -u bench.py --no-cpu-baseline --config c3 --steps 5 --warmup 1 --option pic_poly=1 > gpurun_out/r04b/bench_c3_poly.log 2>&1 || { echo benchc3p_fail; tail -5 gpurun_out/r04b/bench_c3_poly.log; exit 1; }
tail -1 gpurun_out/r04b/bench_c3_poly.log | cut -c1-300
echo r04b_done
