#!/bin/bash
# Lift-splat kernel profile on one GPU box: kernel-trace stats, then one rocprofv3 --pmc pass
# per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass: TCC slots, MI355X guide).
# Output under gpurun_out/pmc_lss/; scripts/pmc_summary.py turns it into profiles/*.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/pmc_lss
mkdir -p $OUT
ARGS="${LSS_ARGS:---batch 8 --iters 20}"
set -o pipefail
timeout -k 10 120 python scripts/bench_lss.py $ARGS > $OUT/bench_lss.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv \
  -- python scripts/bench_lss.py $ARGS > $OUT/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_lss" -d $OUT/fetch -o run \
  --output-format csv -- python scripts/bench_lss.py $ARGS > $OUT/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_lss" -d $OUT/write -o run \
  --output-format csv -- python scripts/bench_lss.py $ARGS > $OUT/write.log 2>&1
rc=$?
cat $OUT/bench_lss.log
exit $rc
