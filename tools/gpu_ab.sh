#!/bin/bash
# A/B of engine options on the C2 bench (run via gpurun), two interleaved rounds:
#   tools/gpu_ab.sh TAG "opt=v ..." "opt=v ..." ...   ("" = the default path)
# Prints per run the realisations/s and the per-launch ms of every kernel group.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=$1; shift
for round in 0 1; do
  i=0
  for set in "$@"; do
    args=""
    for kv in $set; do args="$args --option $kv"; done
    log=gpurun_out/ab_${tag}_${round}_$i.log
    timeout -k 10 300 python bench.py --no-cpu-baseline $args > $log 2>&1 || { echo "fail: $set"; tail -5 $log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print('%-28s %9.0f' % (sys.argv[2], d['value']), {n: v['ms_per_step'] for n,v in k.items() if v.get('launches')})" $log "[$set]"
    i=$((i+1))
  done
done
echo all_ok
