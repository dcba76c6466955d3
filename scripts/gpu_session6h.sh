#!/bin/bash
# Session-6 GPU batch 8: record of HEAD — smoke(), N=2 rehearsal of the multi-rank bench from a
# plain command line (both ranks on device 0, gloo), C5 predict fp16/fp32, C2 line with the
# CPU baseline, C4 lift-splat rocprofv3 summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/s6h
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nn_ops_gpu.py -m gpu -k "squeeze or se_fused" > $O/pytest_se.log 2>&1 || { echo "se pytest failed"; tail -20 $O/pytest_se.log; exit 1; }
tail -1 $O/pytest_se.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
E2EP_PARITY_REPORT=$O/parity_c4.json timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_model_c4_gpu.py -m gpu > $O/pytest_c4.log 2>&1; rc=$?
tail -1 $O/pytest_c4.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1   # 1 = a parity bound failed (numbers recorded); anything else stops
E2EP_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_n2_rehearsal.log 2>&1 || { echo rehearsal failed; tail -20 $O/bench_n2_rehearsal.log; exit 1; }
echo "n2: $(grep -o '"n_gpus": [0-9]*' $O/bench_n2_rehearsal.log | head -1) $(grep -o '"world": {[^}]*}' $O/bench_n2_rehearsal.log | head -1)"
timeout -k 10 300 python scripts/bench_predict.py --precision fp16 --json $O/predict_c5_fp16.json > $O/predict_c5_fp16.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_predict.py --json $O/predict_c5_fp32.json > $O/predict_c5_fp32.log 2>&1 || exit 1
tail -3 $O/predict_c5_fp16.log
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || exit 1
echo "c2: $(grep -o '"value": [0-9.]*' $O/bench_c2.log | head -1) $(grep -o '"cpu_baseline": {"value": [0-9.]*' $O/bench_c2.log)"
timeout -k 10 400 python bench.py --workload c4 --steps 10 --warmup 3 > $O/bench_c4.log 2>&1 || { echo c4 bench failed; tail -5 $O/bench_c4.log; exit 1; }
echo "c4: $(grep -o '"value": [0-9.]*' $O/bench_c4.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c4.log) $(grep -o '"cpu_baseline": {"value": [0-9.]*' $O/bench_c4.log)"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_lss_c4 -o run -- python3 scripts/bench_lss.py --batch 4 --cams 6 --image 512 > $O/bench_lss.log 2>&1 || exit 1
tail -4 $O/bench_lss.log
echo done
