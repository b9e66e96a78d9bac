#!/bin/bash
# A/B of the fused perfect-CSI chain: parity tests, then bench with/without, then kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_doubly_flat.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_parity.log 2>&1 || { echo parity_fail; tail -30 gpurun_out/ab_parity.log; exit 1; }
tail -2 gpurun_out/ab_parity.log
for v in 0 1 2; do
  DSCE_PIC_CHAIN=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/ab_chain$v.log 2>&1 || { echo bench_fail $v; tail -5 gpurun_out/ab_chain$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_chain$v.log').read().strip().splitlines()[-1]); print('chain=$v', round(d['value']), d['kernels_ms'])"
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/ab_stats" -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_prof.log 2>&1 || { echo prof_fail; exit 1; }
echo all_ok
