#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/lp32}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/pytest_conv.log 2>&1; rc=$?; tail -2 $O/pytest_conv.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_conv.log | head -60; exit 1; }
timeout -k 10 500 python scripts/bench_conv.py --precision fp32 --ab "14=1,15=1;14=2,10=11,15=2,13=11;14=2,10=12,15=2,13=12;14=2,10=21,15=2,13=21;14=2,10=22,15=2,13=22" > $O/ab_lp32.txt 2>&1 || exit 1
head -8 $O/ab_lp32.txt
