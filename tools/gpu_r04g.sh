set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04g
timeout -k 10 240 python -u tools/diag/stream_check.py > gpurun_out/r04g/check.log 2>&1 || { echo check_fail; tail -5 gpurun_out/r04g/check.log; exit 1; }
tail -1 gpurun_out/r04g/check.log
for o in pic_stream=0 pic_stream=1 pic_stream=0 pic_stream=1; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 50 --option $o > gpurun_out/r04g/b_$o.log 2>&1 || { echo bench_fail; tail -5 gpurun_out/r04g/b_$o.log; exit 1; }
  echo "$o $(tail -1 gpurun_out/r04g/b_$o.log | cut -c1-160)"
done
