#!/bin/bash
# Row f3: the script's Monte-Carlo runs and Figures 2-5 on the current build
# (run via gpurun from the repo root), written under gpurun_out/results_<TAG>/
# and copied into results/<TAG>/ afterwards.
#   default (C2-C4, 3 schemes, 16384 realisations, with the per-stage NMSE)
#   c5      (BASELINE config 5: 48 x 30, 16 SNR points, 10 048 realisations per point)
#   paper   (script:42-46, FBMC auxiliary, 16384 realisations: Figures 3 / 5)
#   doubly_flat (SimpleVersion_DoublyFlat.m, BASELINE config 1)
# usage: tools/gpu_results.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT/channel-estimation_amd" || exit 1
tag=${1:-x}
out=$GRAFT_REPO_ROOT/gpurun_out/results_$tag
mkdir -p $out/default $out/c5 $out/paper $out/doubly_flat
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m dsce.simulate --config default --reps 16384 --mse --out $out/default/run_default.json --figures $out/default > $out/default/log.txt 2>&1 || { echo default_fail; tail -5 $out/default/log.txt; exit 1; }
tail -1 $out/default/log.txt | cut -c1-300
timeout -k 10 300 python3 -u -m dsce.simulate --config c5 --reps 10048 --mse --out $out/c5/run_c5.json --figures $out/c5 > $out/c5/log.txt 2>&1 || { echo c5_fail; tail -5 $out/c5/log.txt; exit 1; }
tail -1 $out/c5/log.txt | cut -c1-300
timeout -k 10 300 python3 -u -m dsce.simulate --config paper --schemes fbmc_aux --reps 16384 --out $out/paper/run_paper.json --figures $out/paper > $out/paper/log.txt 2>&1 || { echo paper_fail; tail -5 $out/paper/log.txt; exit 1; }
tail -1 $out/paper/log.txt | cut -c1-300
timeout -k 10 300 python3 -u -m dsce.simulate --config doubly_flat --reps 65536 --out $out/doubly_flat/run_doubly_flat.json --figures $out/doubly_flat > $out/doubly_flat/log.txt 2>&1 || { echo flat_fail; tail -5 $out/doubly_flat/log.txt; exit 1; }
tail -1 $out/doubly_flat/log.txt | cut -c1-300
echo results_ok
