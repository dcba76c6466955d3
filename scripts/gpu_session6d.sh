#!/bin/bash
# Session-6 GPU batch 4: A/B of the side-stream weight gradients (E2EP_WGRAD_OVERLAP), per-shape
# conv breakdown (serial), C3 bf16 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/s6d
mkdir -p $O
for i in 1 2; do
  for ov in 0 1; do
    E2EP_WGRAD_OVERLAP=$ov timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_ov${ov}_$i.log 2>&1 || exit 1
    echo "overlap=$ov run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_ov${ov}_$i.log | head -1)"
  done
done
timeout -k 10 300 python scripts/conv_breakdown.py > $O/conv_breakdown.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 > $O/bench_c3_bf16.log 2>&1 || exit 1
echo "bf16: $(grep -o '"value": [0-9.]*' $O/bench_c3_bf16.log | head -1)"
echo done
