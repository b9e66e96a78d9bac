# Bench lines (with CPU baseline) of the given configs on the current source,
# reading the stamped PMC summaries already under profiles/ (gpurun, repo root).
# usage: tools/gpu_lines.sh TAG c3 [c4 ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out/lines_$tag
for c in "$@"; do
  timeout -k 10 600 python3 -u bench.py --config $c > gpurun_out/lines_$tag/$c.log 2> gpurun_out/lines_$tag/$c.err || { echo bench_fail $c; tail -5 gpurun_out/lines_$tag/$c.err; exit 1; }
  tail -1 gpurun_out/lines_$tag/$c.log > gpurun_out/lines_$tag/${c}_bench.json
  cut -c1-150 gpurun_out/lines_$tag/${c}_bench.json
done
echo lines_ok
