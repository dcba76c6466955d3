#!/bin/bash
# Session-6 GPU batch 11: C5 predict kernel profile (fp16, HIP graph), conv variant 0 vs 5 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/s6k
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_predict -o run -- python3 scripts/bench_predict.py --precision fp16 --iters 50 --cpu-iters 0 > $O/predict_prof.log 2>&1 || { echo predict prof failed; tail $O/predict_prof.log; exit 1; }
for i in 1 2; do
  for v in 0 5; do
    E2EP_CONV_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_v${v}_$i.log 2>&1 || exit 1
    echo "variant=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_v${v}_$i.log | head -1)"
  done
done
echo done
