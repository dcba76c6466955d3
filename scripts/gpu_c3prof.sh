#!/bin/bash
# C3 (bf16) step profile + per-shape bf16 / fp32 conv timings on one MI355X.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/c3prof}
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary --precision bf16 > $O/prof.log 2>&1 || exit 1
db=$(find $O/prof -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 120 > $O/step_kernels_c3.txt 2>&1 || true
rm -f $O/prof/*.db
head -3 $O/step_kernels_c3.txt
timeout -k 10 300 python scripts/bench_conv.py --precision bf16 --top 70 > $O/conv_bf16.txt 2>&1 || exit 1
head -3 $O/conv_bf16.txt
timeout -k 10 300 python scripts/bench_conv.py --precision fp32 --top 70 > $O/conv_fp32.txt 2>&1 || exit 1
head -3 $O/conv_fp32.txt
