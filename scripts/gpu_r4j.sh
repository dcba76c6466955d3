#!/bin/bash
# Round 4: branch-capture crash isolation (keep_graph toy, branches without nested forks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4j}
mkdir -p $O
DIAG_VARIANTS=toy_keep,model_cam_nofork,model_heads_nofork timeout -k 10 900 python -u scripts/diag_branch_capture.py > $O/diag_branch.log 2>&1; echo "diag rc $?"
grep -v "^    $" $O/diag_branch.log | tail -60
echo done
