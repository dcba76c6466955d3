#!/bin/bash
# Round 4: BN statistics (tile-major partials, fp32 lane sums, two-level finalize) — tests, C2 / C3 / C4 bench lines, C4 lss timings, step table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4m}
mkdir -p $O
timeout -k 10 200 python scripts/bench_bnstats.py > $O/bnstats.log 2>&1 || { tail -20 $O/bnstats.log; exit 1; }
grep -v amdgpu.ids $O/bnstats.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bn_stats_gpu.py tests/test_lss_gpu.py tests/test_conv_gpu.py -m gpu > $O/pytest_a.log 2>&1; rc=$?
tail -2 $O/pytest_a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_a.log | head -120; exit 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -120; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
echo "c2 $(grep -o '"value": [0-9.]*' $O/c2.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c2.log | head -1)"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --precision bf16 > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
echo "c3 $(grep -o '"value": [0-9.]*' $O/c3.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c3.log | head -1)"
for h in 1; do
  E2EP_TUNE=29=$h timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --workload c4 --steps 10 > $O/c4_h$h.log 2>&1 || { tail -20 $O/c4_h$h.log; exit 1; }
  echo "c4 halves=$h $(grep -o '"value": [0-9.]*' $O/c4_h$h.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c4_h$h.log | head -1) $(grep -o '"lss_c4": {[^}]*}' $O/c4_h$h.log | head -1)"
done
d=$O/prof; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_sequence.py "$db" > $O/step_sequence.txt 2>&1
python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels.txt 2>&1; rm -f $d/*.db
tail -1 $O/step_sequence.txt; head -1 $O/step_kernels.txt
find $O -name "*.csv" -size +2M -delete
echo done
