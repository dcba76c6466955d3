#!/bin/bash
# Round-3 targeted GPU check: new parity tests (captured B=8 step, bf16 C3, host-rig pillar
# index, C4) and the default bench line with its C3/C4/C5 sub-records.
export TMPDIR=/tmp
O=${1:-gpurun_out/r3a}; mkdir -p $O
E2EP_PARITY_REPORT=$O/parity.json timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_train_step_b8_gpu.py tests/test_model_c4_gpu.py tests/test_dataset_gpu.py > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
head -c 3000 $O/bench.log
