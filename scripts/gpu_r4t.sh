#!/bin/bash
# Round 4: 1024-thread BN partial finalize, pipelined lift-splat backward — micro-benchmarks,
# tests, backward A/B against the previous library, C2 with / without epilogue statistics.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4t}
mkdir -p $O
timeout -k 10 200 python scripts/bench_bnstats.py > $O/bnstats.log 2>&1 || { tail -20 $O/bnstats.log; exit 1; }
grep -v amdgpu.ids $O/bnstats.log | head -9
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bn_stats_gpu.py tests/test_lss_gpu.py tests/test_train_step_b8_gpu.py -m gpu > $O/pytest_a.log 2>&1; rc=$?
tail -2 $O/pytest_a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_a.log | head -120; exit 1; }
PREV=e2e-parking-carla_amd/e2ep_amd/libe2ep_hip_prev.so
for r in 1 2; do
  for lib in new prev; do
    if [ $lib = prev ]; then export E2EP_LIB=$PREV; else unset E2EP_LIB; fi
    timeout -k 10 120 python scripts/bench_lss.py --batch 8 --cams 4 --image 256 --iters 50 > $O/c2_${lib}_$r.log 2>&1 || { tail -5 $O/c2_${lib}_$r.log; exit 1; }
    timeout -k 10 120 python scripts/bench_lss.py --batch 4 --cams 6 --image 512 --iters 50 > $O/c4_${lib}_$r.log 2>&1 || { tail -5 $O/c4_${lib}_$r.log; exit 1; }
    echo "== $lib run $r"; grep "lss_bwd" $O/c2_${lib}_$r.log $O/c4_${lib}_$r.log
  done
done
unset E2EP_LIB
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_r$r.log 2>&1 || { tail -20 $O/c2_r$r.log; exit 1; }
  echo "c2 run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_r$r.log | head -1)"
  E2EP_NO_BN_STATS=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_nostats_r$r.log 2>&1 || { tail -20 $O/c2_nostats_r$r.log; exit 1; }
  echo "c2 no-bn-stats run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_nostats_r$r.log | head -1)"
done
echo done
