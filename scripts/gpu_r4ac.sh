#!/bin/bash
# Round 4: block order of the linear paired backward (k_gemm_pair, e2ep_tune key 31: 1 = input
# gradient first, 2 = weight gradient first) — GEMM tests, C2 / C3 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4ac}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_attention_gpu.py -m gpu > $O/pytest_a.log 2>&1; rc=$?
tail -2 $O/pytest_a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_a.log | head -120; exit 1; }
for r in 1 2; do
  for o in 1 2; do
    E2EP_TUNE=31=$o timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2_o${o}_r$r.log 2>&1 || { tail -20 $O/c2_o${o}_r$r.log; exit 1; }
    echo "c2 order=$o run $r $(grep -o '"ms_per_step": [0-9.]*' $O/c2_o${o}_r$r.log | head -1)"
  done
done
for o in 1 2; do
  E2EP_TUNE=31=$o timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --precision bf16 > $O/c3_o$o.log 2>&1 || { tail -20 $O/c3_o$o.log; exit 1; }
  echo "c3 order=$o $(grep -o '"ms_per_step": [0-9.]*' $O/c3_o$o.log | head -1)"
done
echo done
