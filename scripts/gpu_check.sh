#!/bin/bash
# Iteration check on one MI355X: full GPU suite, C2 / C3 bench lines, C2 step kernel table,
# optional extra command ($2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/check}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_gpu.log | head -60; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2.log 2>&1 || exit 1
echo "c2 $(grep -o '"value": [0-9.]*' $O/c2.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c2.log | head -1)"
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --precision bf16 > $O/c3.log 2>&1 || exit 1
echo "c3 $(grep -o '"value": [0-9.]*' $O/c3.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c3.log | head -1)"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $O/prof.log 2>&1 || exit 1
db=$(find $O/prof -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 120 > $O/step_kernels.txt 2>&1; rm -f $O/prof/*.db
head -1 $O/step_kernels.txt
if [ -n "$2" ]; then timeout -k 10 600 bash -c "$2" > $O/extra.txt 2>&1 || exit 1; head -5 $O/extra.txt; fi
echo done
