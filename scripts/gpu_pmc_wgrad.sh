#!/bin/bash
# PMC passes over the six hottest weight-gradient shapes (fp32 C2 kernels), then the bf16 (C3)
# k_wgrad_lp on three of them; summaries under $O/summary_*.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=${1:-gpurun_out/pmc_wgrad}
mkdir -p $O
OUT=$O/fp32 KIND=wgrad SHAPES="stem seg exp160 proj960 exp112 l1" bash scripts/pmc_conv.sh || exit 1
for s in stem seg exp160 proj960 exp112 l1; do python scripts/pmc_table.py $O/fp32 $s; done > $O/summary_fp32.txt 2>&1
E2EP_PRECISION=bf16 OUT=$O/bf16 KIND=wgrad SHAPES="stem seg exp160" bash scripts/pmc_conv.sh || exit 1
for s in stem seg exp160; do python scripts/pmc_table.py $O/bf16 $s; done > $O/summary_bf16.txt 2>&1
find $O -name "*.csv" -size +2M -delete
grep -E "==|utilisation|kernel time|HBM" $O/summary_fp32.txt | head -60
