#!/bin/bash
# A/B of lift-splat kernel variants: parity tests, then the microbench per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lss_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lss_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lss_tests.log
[ $rc -ne 0 ] && exit $rc
for v in ${VARIANTS:-1 2 3}; do
  echo "variant $v"
  E2EP_LSS_FWD=$v timeout -k 10 120 python scripts/bench_lss.py --batch 8 --iters 50 || exit $?
done
