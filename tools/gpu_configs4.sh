#!/bin/bash
# Bench evidence of the current build for the given configurations (stamped PMC
# first, then the line), each via tools/gpu_bench_evidence.sh.
# usage: tools/gpu_configs4.sh TAG c3 [c4 c5 ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-x}
shift
for c in "$@"; do
  # the FBMC / C5 contraction kernel: k_wrow3 (32-row blocks, Opts::wrow) since r04
  bash tools/gpu_bench_evidence.sh ${tag}_$c $c k_wcontract k_wrow3 || { echo config_fail $c; exit 1; }
done
echo configs_ok
