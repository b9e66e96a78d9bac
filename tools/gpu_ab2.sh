#!/bin/bash
# A/B of engine options on the C2 bench in one box (run via gpurun from the repo root):
#   tools/gpu_ab2.sh TAG "opt=v opt2=v" "opt=v'" ...   (each argument one variant; "" = defaults)
# then rocprofv3 kernel stats of the defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
out=gpurun_out/ab_$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for v in "$@"; do
  args=""
  for kv in $v; do args="$args --option $kv"; done
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > $out/v$i.log 2>&1 || { echo "variant $i failed"; tail -5 $out/v$i.log; exit 1; }
  echo "[$v] $(tail -1 $out/v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"], {k: v["ms"] for k, v in d["kernels_ms"].items() if v["ms"]})')"
  i=$((i+1))
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_stats" -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $out/bench_prof.log 2>&1 || { echo prof_fail; exit 1; }
f=$(find $out/prof_stats -name '*kernel_stats.csv' | head -1)
cut -d, -f1-4 "$f" | head -14 | cut -c1-160
echo all_ok
