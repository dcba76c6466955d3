cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r3_gemm && mkdir -p $O &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_conv_gpu.py > $O/pytest_gemm.log 2>&1; tail -2 $O/pytest_gemm.log &&
for i in 1 2; do
E2EP_LIB=$PWD/exp_build/libold.so timeout -k 10 200 python scripts/bench_gemm.py > $O/old_$i.txt 2>&1 || exit 1
timeout -k 10 200 python scripts/bench_gemm.py > $O/new_$i.txt 2>&1 || exit 1
E2EP_LIB=$PWD/exp_build/libold.so timeout -k 10 200 python scripts/bench_conv.py > $O/cold_$i.txt 2>&1 || exit 1
timeout -k 10 200 python scripts/bench_conv.py > $O/cnew_$i.txt 2>&1 || exit 1
done; tail -n1 $O/old_*.txt $O/new_*.txt; grep "conv per step" $O/c*.txt
