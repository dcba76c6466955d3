#!/bin/bash
# PMC passes (MFMA busy, FETCH / WRITE) over the BEV stem and segmentation forward / data
# gradient, fp32 (C2) and bf16 (C3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=${1:-gpurun_out/pmc_stem}
mkdir -p $O
for K in fwd dgrad; do
  OUT=$O/fp32_$K KIND=$K SHAPES="stem seg" bash scripts/pmc_conv.sh || exit 1
  E2EP_PRECISION=bf16 OUT=$O/bf16_$K KIND=$K SHAPES="stem seg" bash scripts/pmc_conv.sh || exit 1
done
for p in fp32 bf16; do for K in fwd dgrad; do for s in stem seg; do python scripts/pmc_table.py $O/${p}_$K $s; done; done; done > $O/summary.txt 2>&1
find $O -name "*.csv" -size +2M -delete
grep -E "==|utilisation|kernel time|HBM" $O/summary.txt | grep -v "k_transpose\|reduce" | head -80
