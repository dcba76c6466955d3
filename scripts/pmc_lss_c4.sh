#!/bin/bash
# Lift-splat at C4 (6 cams x 512^2, B=4) on one GPU box: kernel-trace stats, then separate
# rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE / L2 hit-miss cannot share a pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_lss_c4}
mkdir -p $OUT
ARGS="--batch 4 --cams 6 --image 512 --iters 20"
timeout -k 10 120 python scripts/bench_lss.py $ARGS > $OUT/bench_lss.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv \
  -- python scripts/bench_lss.py $ARGS > $OUT/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_lss" -d $OUT/fetch -o run \
  --output-format csv -- python scripts/bench_lss.py $ARGS > $OUT/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_lss" -d $OUT/write -o run \
  --output-format csv -- python scripts/bench_lss.py $ARGS > $OUT/write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_lss" -d $OUT/l2 -o run \
  --output-format csv -- python scripts/bench_lss.py $ARGS > $OUT/l2.log 2>&1
rc=$?
cat $OUT/bench_lss.log
exit $rc
