# per-level bf16 parity (test failure allowed; fault / timeout ends the run)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/r5v
for L in 2 1; do
  E2EP_BF16_STORE=$L E2EP_PARITY_REPORT=gpurun_out/r5v/par_$L.json timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_train_step_b8_gpu.py -m gpu -k bf16 > gpurun_out/r5v/par_$L.log 2>&1; rc=$?
  echo "level $L rc $rc"; grep "grad_norms" gpurun_out/r5v/par_$L.log
  [ $rc -le 1 ] || exit $rc
done
