#!/bin/bash
# Round 4 iteration box: GPU suite, C2 bench line, replayed-step kernel table, per-shape conv
# timing, the captured-hooks cause diagnostic, stem data-gradient PMC, C4 lift-splat PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
echo "c2 $(grep -o '"value": [0-9.]*' $O/c2.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c2.log | head -1)"
d=$O/prof; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels.txt 2>&1; rm -f $d/*.db
head -1 $O/step_kernels.txt
timeout -k 10 240 python -u scripts/diag_capture_hooks.py > $O/diag_hooks.log 2>&1 || { tail -20 $O/diag_hooks.log; exit 1; }
grep "moved" $O/diag_hooks.log
timeout -k 10 240 python -u scripts/conv_breakdown.py > $O/conv_breakdown.txt 2>&1 || { tail -20 $O/conv_breakdown.txt; exit 1; }
OUT=$O/pmc_stem_dgrad KIND=dgrad SHAPES="stem" bash scripts/pmc_conv.sh || exit 1
python scripts/pmc_table.py $O/pmc_stem_dgrad stem > $O/pmc_stem_dgrad.txt 2>&1
grep -E "==|utilisation|FLOP|kernel time|HBM" $O/pmc_stem_dgrad.txt | head -12
bash scripts/pmc_lss_c4.sh $O/pmc_lss_c4 || exit 1
find $O -name "*.csv" -size +2M -delete
echo done
