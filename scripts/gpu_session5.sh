#!/bin/bash
# Session-5 GPU batch: full GPU suite, C2 / C3 bench lines, attention lane variants (exp_build/
# libraries, correctness + rocprofv3 kernel stats), weight-gradient K-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_all.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_s5.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 > $O/bench_s5_bf16.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/bench_wgrad.py --precisions fp32 bf16 > $O/wgrad_ab.log 2>&1 || exit 1
for L in 1 2 4; do
  lib=e2e-parking-carla_amd/e2ep_amd/libe2ep_hip.so
  [ $L != 1 ] && lib=exp_build/libe2ep_l$L.so
  E2EP_LIB=$PWD/$lib timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_attention_gpu.py -m gpu > $O/attn_l$L.log 2>&1 || exit 1
  E2EP_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/attn_l$L -o run --output-format csv -- python3 scripts/bench_attn.py >> $O/attn_l$L.log 2>&1 || exit 1
done
echo done
