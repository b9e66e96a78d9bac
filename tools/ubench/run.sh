#!/bin/bash
# build + run the issue-cost microbenchmark on the GPU box (gpurun from the repo root)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 tools/ubench/ubench > gpurun_out/ubench.txt 2>&1; rc=$?
cat gpurun_out/ubench.txt
exit $rc
