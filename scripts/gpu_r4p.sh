#!/bin/bash
# Round 4: in-step A/B of the 1x1-conv GEMM route (E2EP_CONV_VARIANT 0 automatic / 4 every 1x1
# forward + data gradient on k_gemm / 5 the same for maps of <= 1024 pixels), two interleaved
# rounds, C2 replayed step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4p}
mkdir -p $O
for r in 1 2; do
  for v in 0 4 5; do
    E2EP_CONV_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_v${v}_r$r.log 2>&1 || { tail -20 $O/c2_v${v}_r$r.log; exit 1; }
    echo "variant $v run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_v${v}_r$r.log | head -1)" | tee -a $O/conv_variant_ab.txt
  done
done
echo done
