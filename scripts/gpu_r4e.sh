#!/bin/bash
# Round 4: model branches on side streams (e2ep_amd.streams): the captured / eager B=8 and C4
# steps and model tests first, then an in-step A/B of E2EP_BRANCH_STREAMS, then the full suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4e}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_step_b8_gpu.py \
  tests/test_model_gpu.py tests/test_model_b8_gpu.py tests/test_graph_gpu.py -m gpu > $O/pytest_model.log 2>&1; rc=$?
tail -2 $O/pytest_model.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error\|Segmentation\|core dumped" $O/pytest_model.log | head -80; exit 1; }
bash scripts/gpu_ab.sh $O/ab E2EP_BRANCH_STREAMS 2 none cam heads cam,heads || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit 1; }
echo done
