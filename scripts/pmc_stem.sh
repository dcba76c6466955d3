#!/bin/bash
# HBM traffic of the BEV stem kernels (scripts/bench_stem.py, B = 8, bf16 operands): one
# rocprofv3 --pmc pass per counter (FETCH_SIZE, WRITE_SIZE), then scripts/pmc_stem_summary.py.
#   bash scripts/pmc_stem.sh OUT_DIR
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_stem}
mkdir -p "$O"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$O/$c" -o run -- python3 scripts/bench_stem.py --iters 5 > "$O/$c.log" 2>&1 || exit 1
done
python3 scripts/pmc_stem_summary.py "$O"
