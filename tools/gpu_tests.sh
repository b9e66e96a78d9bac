#!/bin/bash
# The round-end GPU checks (run via gpurun from the repo root): every -m gpu test,
# then smoke().  Logs under gpurun_out/tests_<TAG>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/tests_${1:-x}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo pytest_fail; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke_fail; tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
echo tests_ok
