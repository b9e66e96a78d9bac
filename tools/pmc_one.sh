#!/bin/bash
# One rocprofv3 counter pass over tools/pmc_probe.py; usage: tools/pmc_one.sh TAG "COUNTERS" [VAR=VAL ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift; ctr=$1; shift
for kv in "$@"; do export "$kv"; done
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc1_$tag" -- python3 tools/pmc_probe.py > gpurun_out/pmc1_$tag.log 2>&1 || { echo "pass failed"; tail -5 gpurun_out/pmc1_$tag.log; exit 1; }
python3 tools/pmc_table.py gpurun_out/pmc1_$tag
