#!/bin/bash
# Round 4: BN statistics from the conv epilogue — new tests, the conv / BN / model suites, C2
# and C3 bench lines, step sequence.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bn_stats_gpu.py tests/test_conv_gpu.py tests/test_splitk_fold_gpu.py -m gpu > $O/pytest_bn.log 2>&1; rc=$?
tail -2 $O/pytest_bn.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_bn.log | head -120; exit 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -120; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
echo "c2 $(grep -o '"value": [0-9.]*' $O/c2.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c2.log | head -1)"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --precision bf16 > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
echo "c3 $(grep -o '"value": [0-9.]*' $O/c3.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c3.log | head -1)"
d=$O/prof; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_sequence.py "$db" > $O/step_sequence.txt 2>&1
python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels.txt 2>&1; rm -f $d/*.db
tail -1 $O/step_sequence.txt; head -1 $O/step_kernels.txt
find $O -name "*.csv" -size +2M -delete
echo done
