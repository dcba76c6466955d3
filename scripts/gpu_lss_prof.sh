#!/bin/bash
# lift-splat microbench + kernel-trace stats (no counters)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/bench_lss.py --batch 8 --iters 50 ${LSS_ARGS} &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/lssprof -o run --output-format csv \
  -- python scripts/bench_lss.py --batch 8 --iters 20 ${LSS_ARGS} > gpurun_out/lssprof.log 2>&1 &&
grep -E "k_lss|k_transpose|k_tile" gpurun_out/lssprof/run_kernel_stats.csv | cut -c1-40,150-
