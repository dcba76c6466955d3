#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/xcd}
mkdir -p $O
E2EP_TUNE=19=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/pytest_conv.log 2>&1; rc=$?; tail -1 $O/pytest_conv.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_conv.log | head -60; exit 1; }
timeout -k 10 300 python scripts/bench_conv.py --precision bf16 --ab "19=1;19=2" > $O/ab_bf16.txt 2>&1 || exit 1
head -12 $O/ab_bf16.txt
BENCH_ARGS="--precision bf16" bash scripts/gpu_ab.sh $O E2EP_TUNE 2 19=1 19=2
