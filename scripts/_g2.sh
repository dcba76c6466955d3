cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_pf &&
E2EP_TUNE=7=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > gpurun_out/r3_pf/pytest_conv_pf3.log 2>&1; tail -2 gpurun_out/r3_pf/pytest_conv_pf3.log &&
timeout -k 10 400 python scripts/bench_conv.py --ab "7=2;7=3" > gpurun_out/r3_pf/ab.txt 2>&1; echo rc=$?; head -4 gpurun_out/r3_pf/ab.txt
