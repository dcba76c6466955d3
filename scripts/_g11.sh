cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r3_tok && mkdir -p $O &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > $O/c2.log 2>&1; echo "c2 $(grep -o '"ms_per_step": [0-9.]*' $O/c2.log | head -1)"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $O/prof.log 2>&1 || exit 1
db=$(find $O/prof -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 200 > $O/step_kernels.txt 2>&1; head -2 $O/step_kernels.txt; grep -c "" $O/step_kernels.txt; grep "at::native\|rocclr\|Cijk" $O/step_kernels.txt
rm -f $O/prof/*.db
