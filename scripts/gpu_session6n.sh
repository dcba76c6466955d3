#!/bin/bash
# Session-6 GPU batch 14: small-grid K splits (E2EP_GEMM_SPLIT_MIN) — GEMM tests with 3, A/B on
# the C2 step (8 = default, 4, 2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/s6n
mkdir -p $O
E2EP_GEMM_SPLIT_MIN=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -n "FAIL\|Error" $O/pytest.log | head; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for v in 8 4 2; do
    E2EP_GEMM_SPLIT_MIN=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_s${v}_$i.log 2>&1 || exit 1
    echo "split_min=$v C2 run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_s${v}_$i.log | head -1)"
  done
done
echo done
