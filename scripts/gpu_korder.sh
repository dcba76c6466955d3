#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/korder}
mkdir -p $O
E2EP_TUNE=18=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/pytest_conv.log 2>&1; rc=$?; tail -1 $O/pytest_conv.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_conv.log | head -60; exit 1; }
timeout -k 10 300 python scripts/bench_conv.py --precision fp32 --ab "18=1;18=2" > $O/ab_fp32.txt 2>&1 || exit 1
head -4 $O/ab_fp32.txt
timeout -k 10 300 python scripts/bench_conv.py --precision bf16 --ab "18=1;18=2" > $O/ab_bf16.txt 2>&1 || exit 1
head -4 $O/ab_bf16.txt
bash scripts/gpu_ab.sh $O E2EP_TUNE 2 18=1 18=2
