#!/bin/bash
# GPU session (run via gpurun from the repo root): the -m gpu tests, the C2
# bench with its CPU baseline, then bench + rocprofv3 kernel stats for C3/C4/C5.
# usage: tools/gpu_configs.sh [tag]   (outputs under gpurun_out/cfg_<tag>/)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-x}
out=gpurun_out/cfg_$tag
mkdir -p $out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo pytest_fail; tail -40 $out/pytest_gpu.log; exit 1; }
  tail -1 $out/pytest_gpu.log
fi
timeout -k 10 400 python -u bench.py > $out/bench_c2.log 2>&1 || { echo bench_fail; tail -20 $out/bench_c2.log; exit 1; }
tail -1 $out/bench_c2.log
for c in ${CONFIGS:-c3 c4 c5}; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $out/bench_$c.log 2>&1 || { echo bench_${c}_fail; tail -20 $out/bench_$c.log; exit 1; }
  tail -1 $out/bench_$c.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_$c" -- python3 bench.py --config $c --no-cpu-baseline --steps 3 --warmup 1 > $out/prof_$c.log 2>&1 || { echo prof_${c}_fail; exit 1; }
done
echo all_ok
