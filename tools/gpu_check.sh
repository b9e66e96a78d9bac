#!/bin/bash
# GPU check (run via gpurun from the repo root): the -m gpu tests, then one bench line.
# usage: tools/gpu_check.sh [pytest selection args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
sel=${@:-tests}
timeout -k 10 900 python -u -m pytest $sel -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_fail; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench_fail; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
echo all_ok
