#!/bin/bash
# Session-6 GPU batch 2: single-launch BN, batched tap-major transposes, SE load ILP —
# full GPU suite, C2 bench line, rocprofv3 kernel trace of the replayed step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/s6b
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_c2.log 2>&1 || exit 1
timeout -k 10 200 python scripts/prof_torch_ops.py > $O/torch_ops.txt 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
db=$(find $O/prof -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 70 > $O/step_kernels.txt 2>&1 || true
tail -1 $O/bench_c2.log | cut -c1-400
echo done
