#!/bin/bash
# Bench line (with its CPU baseline) + counter passes for each non-default
# workload (run via gpurun from the repo root):  tools/gpu_configs.sh TAG c3 c4 c5
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
for cfg in "$@"; do
    out=gpurun_out/cfg_${tag}_$cfg
    mkdir -p $out
    timeout -k 10 400 python -u bench.py --config $cfg > $out/bench.log 2>&1 || { echo bench_fail $cfg; tail -20 $out/bench.log; exit 1; }
    tail -1 $out/bench.log | cut -c1-300
    tools/gpu_pmc_bench.sh ${tag}_$cfg --config $cfg || { echo pmc_fail $cfg; exit 1; }
done
echo configs_ok
