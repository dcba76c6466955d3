#!/bin/bash
# Session-6 GPU batch 15: attention backward split across two streams — full GPU suite, A/B
# (E2EP_ATTN_SPLIT 0 / 1) on the C2 step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/s6o
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -n "FAIL\|Error" $O/pytest_gpu.log | head; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2; do
  for v in 0 1; do
    E2EP_ATTN_SPLIT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_a${v}_$i.log 2>&1 || exit 1
    echo "attn_split=$v C2 run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_a${v}_$i.log | head -1)"
  done
done
echo done
