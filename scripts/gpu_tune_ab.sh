#!/bin/bash
# In-step A/B of the launch-plan tunables (E2EP_TUNE=key=value, see e2ep_tune in include/e2ep.h):
# the defaults against one change at a time (or TUNES="k=v,k=v ..."), interleaved, REPEATS rounds:
#     TUNES="0=1024 0=2048,3=1024" scripts/gpu_tune_ab.sh OUT_DIR REPEATS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/tune}; REP=${2:-2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_nn_ops_gpu.py tests/test_gemm_gpu.py -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -n "FAIL\|Error" $O/pytest.log | head; exit 1; }
tail -1 $O/pytest.log
for i in $(seq 1 $REP); do
  for t in ${TUNES:-0=1024 0=2048 1=8192 2=2048 3=1024 4=1536 5=1024}; do
    log=$O/bench_${t//[=,]/_}_$i.log
    E2EP_TUNE=$t timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $log 2>&1 || exit 1
    echo "tune $t run $i: $(grep -o '"ms_per_step": [0-9.]*' $log | head -1)"
  done
done
echo done
