#!/bin/bash
# One build -> measure iteration on the GPU box (run via gpurun from the repo root):
#   tools/gpu_iter.sh TAG [pytest selection...]
# 1. the selected -m gpu tests (default tests/test_gpu_parity.py)
# 2. one bench line (C2, no CPU leg)
# 3. rocprofv3 kernel stats of a short bench run -> gpurun_out/ks_TAG.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=$1; shift
sel=${@:-tests/test_gpu_parity.py}
timeout -k 10 600 python -u -m pytest $sel -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 || { echo pytest_fail; tail -40 gpurun_out/pytest_$tag.log; exit 1; }
tail -1 gpurun_out/pytest_$tag.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { echo bench_fail; tail -20 gpurun_out/bench_$tag.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', d['roofline']['frac']); print(d['kernels_ms'])" gpurun_out/bench_$tag.log
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$tag" -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/bench_prof_$tag.log 2>&1 || { echo prof_fail; exit 1; }
python3 - "$tag" <<'PY' | tee gpurun_out/ks_$tag.txt
import csv, glob, sys
f = sorted(glob.glob('gpurun_out/prof_%s/**/*_kernel_stats.csv' % sys.argv[1], recursive=True))[-1]
for r in csv.DictReader(open(f)):
    n = r['Name'].replace('dsce::', '').replace('void ', '')
    n = n[:n.index('(')] if '(' in n else n
    print('%-60s %5s %10.1f us %6.2f%%' % (n[:60], r['Calls'], float(r['AverageNs']) / 1e3, float(r['Percentage'])))
PY
echo all_ok
