#!/bin/bash
# Round evidence (run via gpurun from the repo root): all -m gpu tests, smoke,
# the default bench (with its CPU baseline), rocprofv3 kernel stats of the bench
# command, then FETCH_SIZE / WRITE_SIZE passes.  Outputs under gpurun_out/ev_<tag>/.
# usage: tools/gpu_evidence.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/ev_${1:-x}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo pytest_fail; tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke_fail; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { echo bench_fail; tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_stats" -- python3 bench.py --no-cpu-baseline --steps 30 --warmup 5 > $out/bench_prof.log 2>&1 || { echo prof_fail; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_fetch" -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $out/bench_fetch.log 2>&1 || { echo fetch_fail; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_write" -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $out/bench_write.log 2>&1 || { echo write_fail; exit 1; }
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_sq" -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $out/bench_sq.log 2>&1 || { echo sq_fail; exit 1; }
python3 tools/pmc_table.py $out/prof_fetch $out/prof_write $out/prof_sq > $out/table.txt || { echo table_fail; exit 1; }
echo all_ok
