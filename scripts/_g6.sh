cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r3_wg4 && mkdir -p $O &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_gemm_gpu.py > $O/pytest.log 2>&1; tail -2 $O/pytest.log &&
timeout -k 10 400 python scripts/bench_conv.py --ab "9=1,7=1;9=2,7=1" > $O/ab.txt 2>&1; head -3 $O/ab.txt &&
E2EP_LIB=$PWD/exp_build/libold.so timeout -k 10 200 python scripts/bench_conv.py > $O/conv_old.txt 2>&1 && head -2 $O/conv_old.txt &&
timeout -k 10 200 python scripts/bench_gemm.py > $O/gemm.txt 2>&1; tail -1 $O/gemm.txt
