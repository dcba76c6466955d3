#!/bin/bash
# Round-4 record of HEAD on one MI355X: full GPU suite, smoke(), the default bench line (C2 +
# secondary C3 / C4 / C5 + cpu_baseline), rocprofv3 kernel stats of the default bench command,
# fp32 and bf16 replayed-step tables (step_kernels / step_sequence).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4_record}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -n "FAIL\|Error" $O/pytest_gpu.log | head; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
echo "bench: $(grep -o '"value": [0-9.]*' $O/bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/bench.log | head -1)"
d=$O/prof_bench; timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
find $d -name "*kernel_stats.csv" -exec cp {} $O/bench_kernel_stats.csv \;
rm -f $(find $d -name "*.db") $(find $d -name "*kernel_trace.csv")
d=$O/prof; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_sequence.py "$db" > $O/step_sequence_fp32.txt 2>&1
python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels_fp32.txt 2>&1; rm -f $d/*.db
d=$O/prof3; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary --precision bf16 > $d.log 2>&1 || exit 1
db=$(find $d -name "*.db" | tail -n 1); python scripts/step_sequence.py "$db" > $O/step_sequence_bf16.txt 2>&1
python scripts/step_kernels.py "$db" 10 --top 140 > $O/step_kernels_bf16.txt 2>&1; rm -f $d/*.db
tail -1 $O/step_sequence_fp32.txt; tail -1 $O/step_sequence_bf16.txt
find $O -name "*.csv" -size +2M -delete
echo done
