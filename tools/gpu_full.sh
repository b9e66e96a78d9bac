#!/bin/bash
# Full GPU check: gpu tests, smoke, bench, rocprofv3 kernel stats (run via gpurun from the repo root)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_fail; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_fail; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench_fail; exit 1; }
tail -1 gpurun_out/bench.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_stats" -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/bench_prof.log 2>&1 || { echo prof_fail; exit 1; }
echo all_ok
