#!/bin/bash
# Round 4: squeeze-excitation MLP in one per-sample launch each way (k_se_mlp / k_se_mlp_bwd,
# e2ep_tune key 27 = 1) against the two grid-wide launches (key 27 = 3) — nn_ops tests, C2 / C3 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4ad}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_nn_ops_gpu.py tests/test_train_step_b8_gpu.py -m gpu > $O/pytest_a.log 2>&1; rc=$?
tail -2 $O/pytest_a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_a.log | head -120; exit 1; }
for r in 1 2; do
  for v in 1 3; do
    E2EP_TUNE=27=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_s${v}_r$r.log 2>&1 || { tail -20 $O/c2_s${v}_r$r.log; exit 1; }
    echo "c2 se=$v run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_s${v}_r$r.log | head -1)"
  done
done
for v in 1 3; do
  E2EP_TUNE=27=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --precision bf16 > $O/c3_s$v.log 2>&1 || { tail -20 $O/c3_s$v.log; exit 1; }
  echo "c3 se=$v $(grep -o '"ms_per_step": [0-9.]*' $O/c3_s$v.log | head -1)"
done
d=$O/prof; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_sequence.py "$db" > $O/step_sequence.txt 2>&1
python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels.txt 2>&1; rm -f $d/*.db
tail -1 $O/step_sequence.txt; head -1 $O/step_kernels.txt
find $O -name "*.csv" -size +2M -delete
echo done
