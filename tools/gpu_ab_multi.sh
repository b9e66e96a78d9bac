#!/bin/bash
# A/B/C... of several builds of libdsce.so on the C2 bench (run via gpurun from
# the repo root): every ab/*.so copied over the in-tree library in turn (on the
# box's scratch copy only), two interleaved rounds.  tools/gpu_ab_multi.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-x}
lib=channel-estimation_amd/dsce/libdsce.so
cp $lib /tmp/libdsce_intree.so || exit 1
for i in 0 1; do
  for v in ab/*.so; do
    cp $v $lib
    n=$(basename $v .so)
    timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/abm_${tag}_${n}_$i.log 2>&1 || { echo "fail $n"; tail -5 gpurun_out/abm_${tag}_${n}_$i.log; cp /tmp/libdsce_intree.so $lib; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print('%-14s' % sys.argv[2], round(d['value']), {n: v['ms_per_step'] for n,v in k.items() if v.get('launches')})" gpurun_out/abm_${tag}_${n}_$i.log $n
  done
done
cp /tmp/libdsce_intree.so $lib
echo all_ok
