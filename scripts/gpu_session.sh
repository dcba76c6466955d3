#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rehearsal, rocprofv3 kernel-trace profile.
# Every GPU step has its own time limit; a crash / abort / timeout stops the script
# (test failures, rc=1, do not).  STEPS selects the steps; PYTEST_ARGS narrows the tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session.log
  tail -5 "$OUT/$name.log" | tee -a $OUT/session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-pytest,smoke,bench,prof}
PYTEST_ARGS=${PYTEST_ARGS:-tests}
[[ $STEPS == *pytest* ]] && run pytest_gpu 900 python -u -m pytest $PYTEST_ARGS -v -m gpu --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* ]]  && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]]  && run bench 600 python bench.py --steps 20 --warmup 5
[[ $STEPS == *rehearse* ]] && E2EP_BENCH_REHEARSAL=1 run rehearsal_2rank 600 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline
[[ $STEPS == *prof* ]]   && run prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline
[[ $STEPS == *c4prof* ]] && run c4prof 600 rocprofv3 --kernel-trace --stats -d $OUT/c4prof -o run --output-format csv -- python scripts/bench_lss.py --cams 6 --image 512 --batch 4
[[ $STEPS == *pmc* ]]    && run pmc_lss 600 bash scripts/pmc_lss.sh
exit 0
