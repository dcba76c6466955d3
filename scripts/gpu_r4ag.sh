#!/bin/bash
# Round 4: block order of the stride-2 depthwise pair (k_dw_bwd_pair_s2): weight-gradient
# first (HEAD) vs data-gradient first (ab_lib/libe2ep_hip_alt.so via E2EP_LIB) — C2 / C3 A/B
# and the pair kernel's time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4ag}
mkdir -p $O
A=$PWD/ab_lib/libe2ep_hip_alt.so
E2EP_LIB=$A timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_nn_ops_gpu.py -k "pair" -m gpu > $O/pytest_a.log 2>&1; rc=$?
tail -2 $O/pytest_a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_a.log | head -120; exit 1; }
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_w_r$r.log 2>&1 || exit 1
  echo "c2 wgrad-first run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_w_r$r.log | head -1)"
  E2EP_LIB=$A timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_d_r$r.log 2>&1 || exit 1
  echo "c2 dgrad-first run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_d_r$r.log | head -1)"
done
d=$O/prof; E2EP_LIB=$A timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels_alt.txt 2>&1; rm -f $d/*.db
grep "dw_bwd_pair" $O/step_kernels_alt.txt
echo done
