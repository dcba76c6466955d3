#!/bin/bash
# Round 4: C3 paired backward also for the bf16 128 x 128-tile data gradient, run on 128 x 64
# tiles in the pair (k_lp_bwd_pair<2,1,...>) — conv pair tests, C3 / C2 A/B against the
# previous conv_lp (ab_lib/libe2ep_hip_base.so via E2EP_LIB).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4ai}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_gemm_gpu.py tests/test_train_step_b8_gpu.py -m gpu > $O/pytest_a.log 2>&1; rc=$?
tail -2 $O/pytest_a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_a.log | head -120; exit 1; }
B=$PWD/ab_lib/libe2ep_hip_base.so
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --precision bf16 > $O/c3_new_r$r.log 2>&1 || exit 1
  echo "c3 new run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c3_new_r$r.log | head -1)"
  E2EP_LIB=$B timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --precision bf16 > $O/c3_base_r$r.log 2>&1 || exit 1
  echo "c3 base run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c3_base_r$r.log | head -1)"
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_new.log 2>&1 || exit 1
echo "c2 new $(grep -o '"ms_per_step": [0-9.]*' $O/c2_new.log | head -1)"
d=$O/prof3; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary --precision bf16 > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 160 > $O/step_kernels_bf16.txt 2>&1; rm -f $d/*.db
grep "lp_bwd_pair\|k_conv_lp<1" $O/step_kernels_bf16.txt
echo done
