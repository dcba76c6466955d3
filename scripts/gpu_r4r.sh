#!/bin/bash
# Round 4: software-pipelined lift-splat forward — lss tests, then the forward / backward timing
# of the new library against the previous one (E2EP_LIB, built from the last commit) at C2 and
# C4, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4r}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lss_gpu.py -m gpu > $O/pytest_lss.log 2>&1; rc=$?
tail -2 $O/pytest_lss.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_lss.log | head -80; exit 1; }
PREV=e2e-parking-carla_amd/e2ep_amd/libe2ep_hip_prev.so
for r in 1 2; do
  for lib in new prev; do
    if [ $lib = prev ]; then export E2EP_LIB=$PREV; else unset E2EP_LIB; fi
    timeout -k 10 120 python scripts/bench_lss.py --batch 8 --cams 4 --image 256 --iters 50 > $O/c2_${lib}_$r.log 2>&1 || { tail -5 $O/c2_${lib}_$r.log; exit 1; }
    timeout -k 10 120 python scripts/bench_lss.py --batch 4 --cams 6 --image 512 --iters 50 > $O/c4_${lib}_$r.log 2>&1 || { tail -5 $O/c4_${lib}_$r.log; exit 1; }
    echo "== $lib run $r"; grep "lss_" $O/c2_${lib}_$r.log $O/c4_${lib}_$r.log
  done
done
unset E2EP_LIB
echo done
