#!/bin/bash
# Round-end evidence on one MI355X: full GPU suite, smoke, the default bench line (secondary
# configurations + CPU baseline), rocprof step kernel tables for C2 (fp32) and C3 (bf16).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/final}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_gpu.log | head -60; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || exit 1
grep '^{' $O/bench.log | tail -1 | cut -c1-400
for p in fp32 bf16; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$p -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary --precision $p > $O/prof_$p.log 2>&1 || exit 1
  db=$(find $O/prof_$p -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 150 > $O/step_kernels_$p.txt 2>&1; rm -f $O/prof_$p/*.db
  head -1 $O/step_kernels_$p.txt
done
echo done
