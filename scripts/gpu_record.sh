#!/bin/bash
# Record of HEAD on one MI355X: full GPU suite, smoke(), default bench line, C3,
# rocprofv3 kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/record}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -n "FAIL\|Error" $O/pytest_gpu.log | head; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || exit 1
echo "c2: $(grep -o '"value": [0-9.]*' $O/bench_c2.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c2.log | head -1)"
timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 > $O/bench_c3_bf16.log 2>&1 || exit 1
echo "c3: $(grep -o '"value": [0-9.]*' $O/bench_c3_bf16.log | head -1)"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $O/prof.log 2>&1 || exit 1
db=$(find $O/prof -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 80 > $O/step_kernels.txt 2>&1 || true
head -3 $O/step_kernels.txt
echo done
