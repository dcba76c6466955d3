#!/bin/bash
# Round 4: 1x1 paired conv backward (k_conv_bwd_pair1x1: k_conv_gemm data gradient + k_wgrad_1x1)
# — pair tests, C2 A/B over its block order (e2ep_tune key 30) and all conv pairs off, step table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py -k "pair" -m gpu > $O/pytest_a.log 2>&1; rc=$?
tail -2 $O/pytest_a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_a.log | head -120; exit 1; }
for r in 1 2; do
  for v in o1 o2 off; do
    case $v in o1) env="E2EP_TUNE=30=1";; o2) env="E2EP_TUNE=30=2";; off) env="E2EP_CONV_PAIR=0";; esac
    env $env timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_${v}_r$r.log 2>&1 || { tail -20 $O/c2_${v}_r$r.log; exit 1; }
    echo "c2 $v run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_${v}_r$r.log | head -1)"
  done
done
d=$O/prof; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_sequence.py "$db" > $O/step_sequence.txt 2>&1
python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels.txt 2>&1; rm -f $d/*.db
tail -1 $O/step_sequence.txt; head -1 $O/step_kernels.txt
find $O -name "*.csv" -size +2M -delete
echo done
