# which earlier test leaves a sticky HIP error for the next engine's build_mmse
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/diag
for sel in "options_are_validated or default-fbmc_aux" "tx_matrices_on_gpu or default-fbmc_aux" "setup_with_gpu_tx or default-fbmc_aux" "stage_variants or default-fbmc_aux"; do
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_poly.py -x -q --timeout 300 --timeout-method thread -k "$sel" > gpurun_out/diag/s.log 2>&1
  rc=$?
  echo "[$sel] rc=$rc $(tail -1 gpurun_out/diag/s.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
done
