#!/bin/bash
# Session-6 GPU batch 12: skinny GEMM for the decoder's few-row products — GEMM / attention /
# model tests, C5 predict fp16 + fp32, C2 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/s6l
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py tests/test_model_b8_gpu.py -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -n "FAIL\|Error" $O/pytest.log | head; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/bench_predict.py --precision fp16 --json $O/predict_c5_fp16.json > $O/predict_c5_fp16.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_predict.py --json $O/predict_c5_fp32.json > $O/predict_c5_fp32.log 2>&1 || exit 1
python -c "
import json
for f in ['$O/predict_c5_fp16.json','$O/predict_c5_fp32.json']:
    d=json.load(open(f)); print(f, {k:d[k] for k in d if 'p50' in k or 'equal' in k})"
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_c2.log 2>&1 || exit 1
echo "c2: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c2.log | head -1)"
echo done
