#!/bin/bash
# Round 4 end: the full GPU suite and smoke() on HEAD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4_final_check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -n "FAIL\|Error" $O/pytest_gpu.log | head; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
