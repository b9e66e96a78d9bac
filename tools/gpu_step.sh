#!/bin/bash
# One build-measure step on the box (run via gpurun from the repo root):
#   F / K      optional pytest files / -k expression (-m gpu)
#   CONFIG     bench config (default c2); BARGS extra bench args
#   STATS=1    rocprofv3 --kernel-trace --stats of the bench (30 steps), summarised
# Logs under gpurun_out/step_<TAG>/.   usage: tools/gpu_step.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-x}
out=gpurun_out/step_$tag
mkdir -p $out
export TMPDIR=/tmp
cfg=${CONFIG:-c2}
if [ -n "$F" ]; then
  timeout -k 10 900 python -u -m pytest $F ${K:+-k "$K"} -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo pytest_fail; tail -40 $out/pytest_gpu.log; exit 1; }
  tail -1 $out/pytest_gpu.log
fi
if [ "${STATS:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_stats" -- python3 bench.py --config $cfg --no-cpu-baseline --steps 30 --warmup 5 $BARGS > $out/bench_prof.log 2>&1 || { echo prof_fail; tail -5 $out/bench_prof.log; exit 1; }
  python3 - "$out" <<'PY'
import csv, glob, sys
f = sorted(glob.glob('%s/prof_stats/**/*_kernel_stats.csv' % sys.argv[1], recursive=True))[-1]
for r in csv.DictReader(open(f)):
    n = r['Name'].replace('dsce::', '').replace('void ', '')
    n = n[:n.index('(')] if '(' in n else n
    print('%-60s %5s %10.1f us %6.2f%%' % (n[:60], r['Calls'], float(r['AverageNs']) / 1e3, float(r['Percentage'])))
PY
fi
timeout -k 10 400 python3 bench.py --config $cfg --no-cpu-baseline $BARGS > $out/bench.log 2>&1 || { echo bench_fail; tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-400
echo all_ok
