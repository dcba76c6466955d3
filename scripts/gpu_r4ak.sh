#!/bin/bash
# Round 4: stride-2 depthwise pair only up to 131 072 data-gradient units (the 128x128-map layer back on two forked launches)
# — tests, C2 / C3 A/B against HEAD (ab_lib/libe2ep_hip_base.so via E2EP_LIB), kernel times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4ak}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_nn_ops_gpu.py tests/test_train_step_b8_gpu.py -m gpu > $O/pytest_a.log 2>&1; rc=$?
tail -2 $O/pytest_a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_a.log | head -120; exit 1; }
B=$PWD/ab_lib/libe2ep_hip_base.so
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_new_r$r.log 2>&1 || exit 1
  echo "c2 new run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_new_r$r.log | head -1)"
  E2EP_LIB=$B timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_base_r$r.log 2>&1 || exit 1
  echo "c2 base run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_base_r$r.log | head -1)"
done
d=$O/prof; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 160 > $O/step_kernels.txt 2>&1; rm -f $d/*.db
grep "k_dw_" $O/step_kernels.txt
echo done
