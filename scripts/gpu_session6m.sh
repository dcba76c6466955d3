#!/bin/bash
# Session-6 GPU batch 13: skinny GEMM (block per column) — GEMM/model tests, A/B of the row
# limit (0 = off, 16 = decoder at B=1 only, 128 = also the C2 step's 112-row decoder) on C5
# predict and the C2 step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/s6m
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -n "FAIL\|Error" $O/pytest.log | head; exit 1; }
tail -1 $O/pytest.log
for r in 0 16 128; do
  E2EP_GEMM_SKINNY=$r timeout -k 10 300 python scripts/bench_predict.py --precision fp16 --iters 200 --cpu-iters 0 --json $O/predict_fp16_r$r.json > $O/predict_r$r.log 2>&1 || exit 1
  echo "rows<=$r predict fp16: $(python -c "import json;d=json.load(open('$O/predict_fp16_r$r.json'));print(d['graph_p50_ms'])")"
done
for i in 1 2; do
  for r in 0 128; do
    E2EP_GEMM_SKINNY=$r timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_r${r}_$i.log 2>&1 || exit 1
    echo "rows<=$r C2 run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_r${r}_$i.log | head -1)"
  done
done
echo done
