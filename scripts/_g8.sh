cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r3_bw && mkdir -p $O &&
CMD="python3 bench.py --eager --steps 2 --warmup 1 --no-cpu-baseline --no-secondary"
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- $CMD > $O/trace.log 2>&1 || { echo trace failed; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $CMD > $O/fetch.log 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $CMD > $O/write.log 2>&1 || { echo write failed; exit 1; }
python scripts/kernel_bw.py $O/trace $O/fetch $O/write --top 80 > $O/kernel_bw.txt 2>&1; head -50 $O/kernel_bw.txt
rm -rf $O/fetch/*/*agent_info* $O/write/*/*agent_info*
