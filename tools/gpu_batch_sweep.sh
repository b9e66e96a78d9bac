#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rb in 32768 49152 65536 98304 131072 65536; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --reps-per-step $rb --batch $rb > gpurun_out/sw_$rb.log 2>&1 || { echo "fail $rb"; tail -5 gpurun_out/sw_$rb.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],3))" gpurun_out/sw_$rb.log $rb
done
echo all_ok
