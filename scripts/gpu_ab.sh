#!/bin/bash
# In-step A/B of an environment switch on the replayed C2 train step (bench.py, no CPU
# baseline), each value run REPEATS times interleaved:
#     scripts/gpu_ab.sh OUT_DIR VAR REPEATS value1 value2 ...
# e.g. scripts/gpu_ab.sh gpurun_out/ab E2EP_BN_SMALL_LIMITS 3 8192,8192 2048,2048
# (the session-6 A/B results under profiles/r02/session6/*_ab.txt were taken this way; switches
# are listed in INTEGRATION.md §3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$1; VAR=$2; REP=$3; shift 3
mkdir -p "$O"
for i in $(seq 1 "$REP"); do
  for v in "$@"; do
    log="$O/bench_${VAR}_${v//,/_}_$i.log"
    env "$VAR=$v" timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary $BENCH_ARGS > "$log" 2>&1 || exit 1
    echo "$VAR=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' "$log" | head -1)"
  done
done
echo done
