#!/bin/bash
# A/B of engine options on the C2 bench (run via gpurun): tools/gpu_ab.sh TAG "opt=v ..." "opt=v ..." ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=$1; shift
i=0
for set in "$@"; do
  args=""
  for kv in $set; do args="$args --option $kv"; done
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > gpurun_out/ab_${tag}_$i.log 2>&1 || { echo "fail: $set"; tail -5 gpurun_out/ab_${tag}_$i.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-40s %.0f  perfect_ic %.2f ms/launch' % (sys.argv[2], d['value'], d['kernels_ms']['perfect_ic']['ms']/max(1,d['kernels_ms']['perfect_ic']['launches'])))" gpurun_out/ab_${tag}_$i.log "$set"
  i=$((i+1))
done
echo all_ok
