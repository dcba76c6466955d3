cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r3_c3 && mkdir -p $O &&
E2EP_PARITY_REPORT=$O/parity.json timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_train_step_b8_gpu.py tests/test_model_gpu.py > $O/pytest.log 2>&1; rc=$?; grep -E "passed|failed" $O/pytest.log | tail -2; grep -A3 "bf16_train_b8 loss\|grad_norms" $O/pytest.log | head -12; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --precision bf16 > $O/c3.log 2>&1; echo "c3 $(grep -o '"ms_per_step": [0-9.]*' $O/c3.log | head -1)"
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2.log 2>&1; echo "c2 $(grep -o '"ms_per_step": [0-9.]*' $O/c2.log | head -1)"
