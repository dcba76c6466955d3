cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_conv &&
timeout -k 10 200 python scripts/bench_conv.py --top 45 > gpurun_out/r3_conv/bench_conv.txt 2>&1 &&
OUT=gpurun_out/r3_conv/pmc SHAPES="exp160 proj960 up216 l1" timeout -k 10 700 bash scripts/pmc_conv.sh > gpurun_out/r3_conv/pmc.log 2>&1 &&
for s in exp160 proj960 up216 l1; do python scripts/pmc_table.py gpurun_out/r3_conv/pmc $s; done > gpurun_out/r3_conv/pmc_summary.txt 2>&1; echo rc=$?
