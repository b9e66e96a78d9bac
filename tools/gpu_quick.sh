#!/bin/bash
# GPU quick check (run via gpurun from the repo root): selected -m gpu tests
# (pytest -k expression in $K, file list in $F), then one bench line per config
# in $CONFIGS (default c2) with extra bench args $BARGS.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$F" ]; then
  timeout -k 10 900 python -u -m pytest $F ${K:+-k "$K"} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_fail; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
for c in ${CONFIGS:-c2}; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline $BARGS > gpurun_out/bench_$c.log 2>&1 || { echo bench_fail; tail -20 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log
done
echo all_ok
