#!/bin/bash
# usage: tools/ab_env.sh "ENV=VAL ..." "ENV=VAL ..." ...  — parity (C2 + channel tests) then one bench per env set
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_doubly_flat.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_parity.log 2>&1 || { echo parity_fail; tail -30 gpurun_out/ab_parity.log; exit 1; }
tail -1 gpurun_out/ab_parity.log
i=0
for set in "$@"; do
  i=$((i+1))
  env $set timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/ab_env$i.log 2>&1 || { echo bench_fail "$set"; tail -5 gpurun_out/ab_env$i.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_env$i.log').read().strip().splitlines()[-1]); print('[$set]', round(d['value']), {k: round(v['ms']/v['launches'],3) for k,v in d['kernels_ms'].items()})"
done
echo all_ok
