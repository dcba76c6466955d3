#!/bin/bash
# Round 4: in-step A/B of the fused squeeze-excitation (tune 27) and the split-K folds
# (tune 28), and the replayed step's kernel table with both on / both off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4b}
mkdir -p $O
bash scripts/gpu_ab.sh $O/ab E2EP_TUNE 2 27=2,28=2 27=1 28=1 27=1,28=1 || exit 1
for t in 27=2,28=2 27=1,28=1; do
  d=$O/prof_${t//[=,]/_}
  E2EP_TUNE=$t timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary > $d.log 2>&1 || exit 1
  db=$(find $d -name "*.db" | tail -n 1); python scripts/step_kernels.py "$db" 10 --top 140 > $d.txt 2>&1; rm -f $d/*.db
  head -1 $d.txt
done
echo done
