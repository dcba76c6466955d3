#!/bin/bash
# Session-6 GPU batch: HEAD check in a fresh container — full GPU suite, default bench line
# (C2 with the CPU baseline), C3 bf16 line, rocprofv3 kernel trace of the replayed step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/s6
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 > $O/bench_c3_bf16.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
db=$(find $O/prof -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 70 > $O/step_kernels.txt 2>&1 || true
echo done
