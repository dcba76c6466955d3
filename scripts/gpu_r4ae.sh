#!/bin/bash
# Round 4: depthwise backward pairs incl. stride 2 (k_dw_bwd_pair_s2) — tests, C2 / C3 A/B against E2EP_DW_PAIR=0.
# C2 / C3 A/B against the forked two-launch form (E2EP_DW_PAIR=0), step table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4ae}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_nn_ops_gpu.py -k "pair or depthwise" -m gpu > $O/pytest_a.log 2>&1; rc=$?
tail -2 $O/pytest_a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_a.log | head -120; exit 1; }
for r in 1 2; do
  for pr in 1 0; do
    E2EP_DW_PAIR=$pr timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_p${pr}_r$r.log 2>&1 || { tail -20 $O/c2_p${pr}_r$r.log; exit 1; }
    echo "c2 pair=$pr run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_p${pr}_r$r.log | head -1)"
  done
done
for pr in 1 0 1 0; do
  E2EP_DW_PAIR=$pr timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --precision bf16 > $O/c3_p$pr.log 2>&1 || { tail -20 $O/c3_p$pr.log; exit 1; }
  echo "c3 pair=$pr $(grep -o '"ms_per_step": [0-9.]*' $O/c3_p$pr.log | head -1)"
done
find $O -name "*.csv" -size +2M -delete
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -120; exit 1; }
echo done
