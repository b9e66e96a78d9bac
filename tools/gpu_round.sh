#!/bin/bash
# Round-end GPU evidence (run via gpurun from the repo root): gpu tests, smoke,
# bench, rocprofv3 kernel stats of the bench, FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_fail; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_fail; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench_fail; tail -5 gpurun_out/bench.log; exit 1; }
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_stats" -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/bench_prof.log 2>&1 || { echo prof_fail; exit 1; }
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fetch" -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/bench_fetch.log 2>&1 || { echo fetch_fail; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_write" -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/bench_write.log 2>&1 || { echo write_fail; exit 1; }
echo all_ok
