#!/bin/bash
# Round 4 iteration box: the full GPU suite (new: C4 B=4 captured step, device-rig pillar
# index, split-K folds, fused squeeze-excitation), the captured-hooks diagnostic with the
# warm-up weight check, a C2 bench line, per-shape conv timing and the stem data-gradient PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
echo "c2 $(grep -o '"value": [0-9.]*' $O/c2.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c2.log | head -1)"
timeout -k 10 240 python -u scripts/diag_capture_hooks.py CN > $O/diag_CN.log 2>&1 || { tail -20 $O/diag_CN.log; exit 1; }
grep "CN:" $O/diag_CN.log
timeout -k 10 240 python -u scripts/conv_breakdown.py > $O/conv_breakdown.txt 2>&1 || { tail -20 $O/conv_breakdown.txt; exit 1; }
OUT=$O/pmc_stem_dgrad KIND=dgrad SHAPES="stem" bash scripts/pmc_conv.sh || exit 1
python scripts/pmc_table.py $O/pmc_stem_dgrad stem > $O/pmc_stem_dgrad.txt 2>&1
grep -E "==|utilisation|FLOP|kernel time|HBM" $O/pmc_stem_dgrad.txt | head -20
find $O -name "*.csv" -size +2M -delete
echo done
