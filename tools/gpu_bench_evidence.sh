#!/bin/bash
# Bench evidence of one source build (run via gpurun from the repo root), in the
# order that stamps the line with this build's own counters:
#   1. rocprofv3 kernel stats of the bench command (30 steps),
#   2. separate --pmc passes: FETCH_SIZE, WRITE_SIZE, the SQ counters,
#   3. tools/prof_summary.py writes profiles/<TAG>_pmc_all.json (every kernel
#      group) and profiles/<TAG>_pmc_<dominant>.json, stamped with the source hash,
#   4. bench.py (default: C2 with its CPU baseline) reads them: the line carries
#      traffic / limiter / per-kernel counters of THIS build.
# Outputs under gpurun_out/ev_<TAG>/ (profiles/<TAG>_* copied there too).
# usage: tools/gpu_bench_evidence.sh TAG [CONFIG] [BENCH_KERNEL] [KERNEL_SUBSTR] [extra bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-x}
cfg=${2:-c2}
bk=${3:-k_mic_data}
ks=${4:-k_mic_data}
shift 4 2>/dev/null
out=gpurun_out/ev_${tag}
mkdir -p "$out"
export TMPDIR=/tmp
pb="python3 bench.py --config $cfg --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_stats" -- $pb --steps 30 --warmup 5 "$@" > $out/bench_prof.log 2>&1 || { echo prof_fail; tail -5 $out/bench_prof.log; exit 1; }
echo stats_ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_fetch" -- $pb --steps 2 --warmup 1 "$@" > $out/bench_fetch.log 2>&1 || { echo fetch_fail; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_write" -- $pb --steps 2 --warmup 1 "$@" > $out/bench_write.log 2>&1 || { echo write_fail; exit 1; }
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/prof_sq" -- $pb --steps 2 --warmup 1 "$@" > $out/bench_sq.log 2>&1 || { echo sq_fail; exit 1; }
echo pmc_ok
python3 tools/prof_summary.py --all "$tag" $out/prof_stats $out/prof_fetch $out/prof_write "$cfg" $out/prof_sq > $out/pmc_all.json || { echo summary_all_fail; exit 1; }
python3 tools/prof_summary.py "$tag" $out/prof_stats $out/prof_fetch $out/prof_write "$ks" "$bk" "$cfg" $out/prof_sq > $out/pmc_one.json || { echo summary_fail; exit 1; }
python3 tools/pmc_table.py $out/prof_fetch $out/prof_write $out/prof_sq > $out/table.txt 2>&1 || true
timeout -k 10 600 python3 -u bench.py --config "$cfg" "$@" > $out/bench.log 2> $out/bench.err || { echo bench_fail; tail -20 $out/bench.err; exit 1; }
tail -1 $out/bench.log > $out/bench_line.json
cp profiles/${tag}_* $out/ 2>/dev/null
cut -c1-600 $out/bench_line.json
echo all_ok
