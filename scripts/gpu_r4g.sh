#!/bin/bash
# Round 4: branch-capture crash stack (faulthandler), GEMM split-min A/B on the C2 step with
# the in-launch fold, launch-by-launch step sequence.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4g}
mkdir -p $O
for sm in 8 4 2; do
  E2EP_GEMM_SPLIT_MIN=$sm timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_sm$sm.log 2>&1 || { tail -20 $O/c2_sm$sm.log; exit 1; }
  echo "split_min $sm $(grep -o '"value": [0-9.]*' $O/c2_sm$sm.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c2_sm$sm.log | head -1)"
done
d=$O/prof; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_sequence.py "$db" > $O/step_sequence.txt 2>&1
python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels.txt 2>&1; rm -f $d/*.db
tail -1 $O/step_sequence.txt; head -1 $O/step_kernels.txt
find $O -name "*.csv" -size +2M -delete
DIAG_VARIANTS=model_cam timeout -k 10 900 python -u scripts/diag_branch_capture.py > $O/diag_branch.log 2>&1; echo "diag rc $?"
tail -100 $O/diag_branch.log
echo done
