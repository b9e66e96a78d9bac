# Round-end evidence of the final source: every GPU test + smoke, then the C2
# bench evidence (stamped PMC first).  usage: tools/gpu_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-final}
out=gpurun_out/tests_$tag
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo pytest_fail; tail -30 $out/pytest_gpu.log; exit 1; }
grep -n "dsce_destroy:\|stale HIP" $out/pytest_gpu.log | head -3
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke_fail; tail -10 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
bash tools/gpu_bench_evidence.sh $tag c2 k_mic_data k_mic_data
