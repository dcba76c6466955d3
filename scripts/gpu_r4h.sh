#!/bin/bash
# Round 4: fork threshold A/B (E2EP_FORK_MIN_US) on the C2 step, side-stream tests, and the
# step sequence at the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4h}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_attention_gpu.py -m gpu -k "side_stream or split or overlap" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for us in 0 10 20 40 80 1000000; do
  E2EP_FORK_MIN_US=$us timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_us$us.log 2>&1 || { tail -20 $O/c2_us$us.log; exit 1; }
  echo "fork_min_us $us $(grep -o '"value": [0-9.]*' $O/c2_us$us.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c2_us$us.log | head -1)"
done
for us in 0 20 1000000; do
  E2EP_FORK_MIN_US=$us timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --precision bf16 > $O/c3_us$us.log 2>&1 || { tail -20 $O/c3_us$us.log; exit 1; }
  echo "c3 fork_min_us $us $(grep -o '"value": [0-9.]*' $O/c3_us$us.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/c3_us$us.log | head -1)"
done
d=$O/prof; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_sequence.py "$db" > $O/step_sequence.txt 2>&1
python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels.txt 2>&1; rm -f $d/*.db
tail -1 $O/step_sequence.txt; head -1 $O/step_kernels.txt
find $O -name "*.csv" -size +2M -delete
echo done
