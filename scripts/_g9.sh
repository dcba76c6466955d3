cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r3_dw2 && mkdir -p $O &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nn_ops_gpu.py tests/test_model_gpu.py > $O/pytest.log 2>&1; tail -1 $O/pytest.log &&
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/new_$i.log 2>&1 || exit 1
echo "new $i $(grep -o '"ms_per_step": [0-9.]*' $O/new_$i.log | head -1)"
done
CMD="python3 bench.py --eager --steps 2 --warmup 1 --no-cpu-baseline --no-secondary"
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- $CMD > $O/trace.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $CMD > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $CMD > $O/write.log 2>&1 || exit 1
python scripts/kernel_bw.py $O/trace $O/fetch $O/write --match "k_dw|k_bn|k_se" > $O/kernel_bw.txt 2>&1; cat $O/kernel_bw.txt
