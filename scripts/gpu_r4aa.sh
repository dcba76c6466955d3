#!/bin/bash
# Round 4: block order of the paired conv backward (e2ep_tune key 29: 1 = data-gradient blocks
# first, 2 = weight-gradient blocks first) — pair tests in both orders, C2 / C3 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4aa}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py -k "pair" -m gpu > $O/pytest_a.log 2>&1; rc=$?
tail -2 $O/pytest_a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_a.log | head -120; exit 1; }
for r in 1 2; do
  for o in 1 2; do
    E2EP_TUNE=29=$o timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_o${o}_r$r.log 2>&1 || { tail -20 $O/c2_o${o}_r$r.log; exit 1; }
    echo "c2 order=$o run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_o${o}_r$r.log | head -1)"
  done
done
for r in 1 2; do
  for o in 1 2; do
    E2EP_TUNE=29=$o timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --precision bf16 > $O/c3_o${o}_r$r.log 2>&1 || { tail -20 $O/c3_o${o}_r$r.log; exit 1; }
    echo "c3 order=$o run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c3_o${o}_r$r.log | head -1)"
  done
done
d=$O/prof; E2EP_TUNE=29=2 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels_o2.txt 2>&1; rm -f $d/*.db
find $O -name "*.csv" -size +2M -delete
echo done
