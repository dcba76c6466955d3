#!/bin/bash
# Achieved HBM bandwidth of the BN / depthwise / SE / layout kernels in the eager C2 train step:
# one kernel-trace run (durations) and one FETCH_SIZE and one WRITE_SIZE counter pass, each its
# own rocprofv3 run, then scripts/kernel_bw.py joins them (MI355X_MICROARCH.md HBM recipe).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
export E2EP_WGRAD_OVERLAP=0  # weight gradients serial: each kernel timed alone
O=${1:-gpurun_out/kbw}
mkdir -p $O
CMD="bench.py --eager --steps 3 --warmup 2 --no-cpu-baseline --no-secondary"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/T -o run --output-format csv -- python3 $CMD > $O/t.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/F -o run --output-format csv -- python3 $CMD > $O/f.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/W -o run --output-format csv -- python3 $CMD > $O/w.log 2>&1 || exit 1
python scripts/kernel_bw.py $O/T $O/F $O/W --match 'k_bn_|k_dw_|k_se_|k_cat_|k_add_f32|k_rng|k_transpose' --top 60 > $O/kernel_bw.txt 2>&1
rm -rf $O/T $O/F $O/W
head -40 $O/kernel_bw.txt
