#!/bin/bash
# Round 4: lift-splat lane schedule (C4) + GEMM / workspace tests, C4 lift-splat PMC, C4 and
# C2 bench lines, replayed-step grid-fill table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4d}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lss_gpu.py \
  tests/test_gemm_gpu.py tests/test_splitk_fold_gpu.py tests/test_model_c4_gpu.py -m gpu > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit 1; }
bash scripts/pmc_lss_c4.sh $O/pmc_lss_c4 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --workload c4 --steps 10 > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
echo "c4 $(grep -o '"value": [0-9.]*' $O/c4.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c4.log | head -1)"
d=$O/prof; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels.txt 2>&1
python scripts/step_grid.py "$db" 10 > $O/step_grid.txt 2>&1; rm -f $d/*.db
head -1 $O/step_kernels.txt; head -12 $O/step_grid.txt
find $O -name "*.csv" -size +2M -delete
echo done
