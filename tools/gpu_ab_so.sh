#!/bin/bash
# A/B of two builds of libdsce.so on the C2 bench (run via gpurun from the repo
# root): the in-tree library, then ab/libdsce_alt.so copied over it (on the box's
# scratch copy only), alternating twice.  tools/gpu_ab_so.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-x}
lib=channel-estimation_amd/dsce/libdsce.so
cp $lib /tmp/libdsce_base.so || exit 1
for i in 0 1; do
  for v in base alt; do
    if [ $v = base ]; then cp /tmp/libdsce_base.so $lib; else cp ab/libdsce_alt.so $lib; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_${tag}_${v}_$i.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/ab_${tag}_${v}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print(sys.argv[2], round(d['value']), {n: v['ms_per_step'] for n,v in k.items() if v.get('launches')})" gpurun_out/ab_${tag}_${v}_$i.log $v
  done
done
cp /tmp/libdsce_base.so $lib
echo all_ok
