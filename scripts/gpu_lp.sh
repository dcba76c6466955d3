#!/bin/bash
# k_conv_lp: conv GPU tests, then per-shape bf16 timings of the new kernel (11=2) vs the
# fp32-era kernels with bf16 operands (11=1), then the C3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/lp}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/pytest_conv.log 2>&1; rc=$?; tail -3 $O/pytest_conv.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_conv.log | head -60; exit 1; }
timeout -k 10 400 python scripts/bench_conv.py --precision bf16 --ab "11=1,12=1;11=2,12=2,16=32,17=32;11=2,12=2;11=2,12=2,17=128" > $O/ab_lp.txt 2>&1 || exit 1
head -60 $O/ab_lp.txt
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --precision bf16 > $O/c3.log 2>&1 || exit 1
echo "c3 $(grep -o '"value": [0-9.]*' $O/c3.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c3.log | head -1)"
