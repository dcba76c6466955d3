#!/bin/bash
# Session-6 GPU batch 10: full GPU suite (incl. C4 parity, SE small planes), C2 bench, step
# kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/s6j
mkdir -p $O
E2EP_PARITY_REPORT=$O/parity.json timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -n "FAIL\|Error" $O/pytest_gpu.log | head; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_c2.log 2>&1 || exit 1
echo "c2: $(grep -o '"value": [0-9.]*' $O/bench_c2.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c2.log | head -1)"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
db=$(find $O/prof -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 80 > $O/step_kernels.txt 2>&1 || true
grep "k_se_" $O/step_kernels.txt
echo done
