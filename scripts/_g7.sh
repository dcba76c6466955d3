cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r3_step && mkdir -p $O &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/pytest.log 2>&1; tail -1 $O/pytest.log &&
for i in 1 2; do
E2EP_LIB=$PWD/exp_build/libold.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/old_$i.log 2>&1 || exit 1
echo "old $i $(grep -o '"ms_per_step": [0-9.]*' $O/old_$i.log | head -1)"
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/new_$i.log 2>&1 || exit 1
echo "new $i $(grep -o '"ms_per_step": [0-9.]*' $O/new_$i.log | head -1)"
E2EP_TUNE=9=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/new1_$i.log 2>&1 || exit 1
echo "new wgrad1 $i $(grep -o '"ms_per_step": [0-9.]*' $O/new1_$i.log | head -1)"
done
