cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r3_seg && mkdir -p $O &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > $O/bench.log 2>&1; grep -o '"value": [0-9.]*' $O/bench.log | head -1
