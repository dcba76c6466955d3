#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/attn_lanes}
mkdir -p $O
for v in 2 4; do
  E2EP_TUNE=20=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $O/pytest_attn_$v.log 2>&1 || { tail -30 $O/pytest_attn_$v.log; exit 1; }
  tail -1 $O/pytest_attn_$v.log
done
bash scripts/gpu_ab.sh $O E2EP_TUNE 2 20=1 20=2 20=4 || exit 1
