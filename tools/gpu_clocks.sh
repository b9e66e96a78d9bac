#!/bin/bash
# GPU clock / power while the C2 bench runs (gpurun from the repo root): rocm-smi
# samples every ~0.5 s in the background, bench with many steps in the foreground.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/clk
( for i in $(seq 1 80); do date +%s.%N; rocm-smi --showclocks --showpower 2>&1 | grep -E "sclk|fclk|mclk|Power|W" ; sleep 0.4; done ) > gpurun_out/clk/smi.txt 2>&1 &
SMI=$!
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 1500 --warmup 2 > gpurun_out/clk/bench.log 2>&1; rc=$?
kill $SMI 2>/dev/null
tail -1 gpurun_out/clk/bench.log | cut -c1-200
grep -E "sclk" gpurun_out/clk/smi.txt | sort | uniq -c | sort -rn | head -12
grep -iE "power" gpurun_out/clk/smi.txt | sort | uniq -c | sort -rn | head -12
exit $rc
