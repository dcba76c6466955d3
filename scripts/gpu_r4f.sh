#!/bin/bash
# Round 4: which side-stream branch captures crash hipStreamEndCapture; then (branches off) the
# full suite with the own-executable graph launches, and a C2 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4f}
mkdir -p $O
timeout -k 10 900 python -u scripts/diag_branch_capture.py > $O/diag_branch.log 2>&1; echo "diag rc $?"
cat $O/diag_branch.log
export E2EP_BRANCH_STREAMS=none
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
echo "c2 $(grep -o '"value": [0-9.]*' $O/c2.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c2.log | head -1)"
echo done
