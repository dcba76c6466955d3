#!/bin/bash
# Round 4: single-launch finalize of the BN partials — micro-benchmark, BN / model tests, C2 / C3
# bench lines, step table; then the in-step 1x1-conv route A/B (gpu_r4p.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4q}
mkdir -p $O
timeout -k 10 200 python scripts/bench_bnstats.py > $O/bnstats.log 2>&1 || { tail -20 $O/bnstats.log; exit 1; }
grep -v amdgpu.ids $O/bnstats.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bn_stats_gpu.py tests/test_train_step_b8_gpu.py tests/test_model_b8_gpu.py -m gpu > $O/pytest_a.log 2>&1; rc=$?
tail -2 $O/pytest_a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_a.log | head -120; exit 1; }
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_r$r.log 2>&1 || { tail -20 $O/c2_r$r.log; exit 1; }
  echo "c2 run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_r$r.log | head -1)"
  E2EP_NO_BN_STATS=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_nostats_r$r.log 2>&1 || { tail -20 $O/c2_nostats_r$r.log; exit 1; }
  echo "c2 no-bn-stats run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_nostats_r$r.log | head -1)"
done
d=$O/prof; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_sequence.py "$db" > $O/step_sequence.txt 2>&1
python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels.txt 2>&1; rm -f $d/*.db
tail -1 $O/step_sequence.txt; head -1 $O/step_kernels.txt
find $O -name "*.csv" -size +2M -delete
bash scripts/gpu_r4p.sh gpurun_out/r4p
echo done
