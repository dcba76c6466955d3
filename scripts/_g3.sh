cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r3_tiles &&
timeout -k 10 700 python scripts/bench_conv.py --ab "v=0,8=1,9=1;v=2,8=1,9=1;v=1,8=64128,9=1;v=1,8=64064,9=1;v=1,8=1,9=2;v=1,8=32128,9=1;v=1,8=64128,9=2" > gpurun_out/r3_tiles/ab.txt 2>&1; echo rc=$?; head -9 gpurun_out/r3_tiles/ab.txt
