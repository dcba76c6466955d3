#!/bin/bash
# Round 4: fp32 K order per conv shape (tap outer vs channel-chunk outer) in isolation, and the
# BEV stem forward's HBM fetch under each order (23x re-reads, tap-outer).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/r4n}
mkdir -p $O
timeout -k 10 400 python scripts/bench_conv.py --ab "18=3;18=2" --top 60 > $O/korder_ab_fp32.txt 2>&1 || { tail -20 $O/korder_ab_fp32.txt; exit 1; }
head -12 $O/korder_ab_fp32.txt
for k in 3 2; do
  E2EP_TUNE=18=$k OUT=$O/stem_fwd_k$k KIND=fwd SHAPES="stem" bash scripts/pmc_conv.sh > $O/pmc_k$k.log 2>&1 || { tail -20 $O/pmc_k$k.log; exit 1; }
  python scripts/pmc_table.py $O/stem_fwd_k$k stem > $O/stem_fwd_k$k.txt 2>&1
  grep -E "==|utilisation|kernel time|HBM" $O/stem_fwd_k$k.txt | head -20
done
find $O -name "*.csv" -size +2M -delete
echo done
