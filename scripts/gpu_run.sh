#!/bin/bash
# One parametrised GPU driver for gpurun (replaces the round-4 one-off gpu_r4*.sh scripts).
#   scripts/gpu_run.sh OUT_DIR STEP [STEP ...]
# Steps run in order, each under its own time limit, and the script stops at the first failure:
#   tests[:FILES]     GPU tests (all of tests/, or the comma-separated files)
#   smoke             __graft_entry__.smoke()
#   bench             the default bench line (C2 + secondary C3 / C4 / C5 + cpu_baseline)
#   c2 | c3           one bench line, no CPU baseline / secondaries (c3: --precision bf16)
#   ab:VAR:REP:v1,v2  interleaved in-step A/B of an environment switch on C2 (c3ab: on C3);
#                     values separated by '/' when they contain commas, by '|' when they
#                     contain '/' (library paths for E2EP_LIB)
#   table:PREC        rocprofv3 kernel trace of 10 replayed steps (PREC fp32 | bf16) ->
#                     step_kernels_PREC.txt + step_sequence_PREC.txt
#   stats             rocprofv3 --kernel-trace --stats of the default bench command
#   cmd:SHELL         an extra command (e.g. a scripts/*.py micro-benchmark), 600 s limit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$1; shift
mkdir -p "$O"
val() { grep -o "\"$1\": [0-9.]*" "$2" | head -1; }
for st in "$@"; do
  case "$st" in
    tests*)
      files=tests; [ "$st" != tests ] && files=$(echo "${st#tests:}" | tr ',' ' ')
      timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread $files -m gpu > "$O/pytest.log" 2>&1; rc=$?
      tail -2 "$O/pytest.log"
      [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" "$O/pytest.log" | head -120; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 400 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
      echo "bench $(val value "$O/bench.log") $(val ms_per_step "$O/bench.log")" ;;
    c2|c3)
      p=""; [ "$st" = c3 ] && p="--precision bf16"
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary $p > "$O/$st.log" 2>&1 || { tail -20 "$O/$st.log"; exit 1; }
      echo "$st $(val value "$O/$st.log") $(val ms_per_step "$O/$st.log")" ;;
    ab:*|c3ab:*)
      IFS=: read -r kind var rep vals <<< "$st"
      p=""; [ "$kind" = c3ab ] && p="--precision bf16"
      sep=','; [[ "$vals" == */* ]] && sep='/'; [[ "$vals" == *"|"* ]] && sep='|'
      IFS="$sep" read -r -a vs <<< "$vals"
      for i in $(seq 1 "$rep"); do
        for v in "${vs[@]}"; do
          tag=${v//,/_}; tag=${tag//\//_}; log="$O/${kind}_${var}_${tag}_$i.log"
          env "$var=$v" timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary $p > "$log" 2>&1 || { tail -20 "$log"; exit 1; }
          echo "$kind $var=$v run $i: $(val ms_per_step "$log")"
        done
      done ;;
    table:*)
      prec=${st#table:}; d=$O/prof_$prec
      timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$d" -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-secondary --precision "$prec" > "$d.log" 2>&1 || { tail -20 "$d.log"; exit 1; }
      db=$(find "$d" -name "*.db" | tail -n 1)
      python scripts/step_sequence.py "$db" > "$O/step_sequence_$prec.txt" 2>&1
      python scripts/step_kernels.py "$db" 10 --top 160 > "$O/step_kernels_$prec.txt" 2>&1
      rm -f $(find "$d" -name "*.db")
      tail -1 "$O/step_sequence_$prec.txt"; head -1 "$O/step_kernels_$prec.txt" ;;
    stats)
      d=$O/prof_bench
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- python3 bench.py > "$d.log" 2>&1 || { tail -20 "$d.log"; exit 1; }
      find "$d" -name "*kernel_stats.csv" -exec cp {} "$O/bench_kernel_stats.csv" \;
      rm -f $(find "$d" -name "*.db") $(find "$d" -name "*kernel_trace.csv") ;;
    cmd:*)
      timeout -k 10 600 bash -c "${st#cmd:}" > "$O/extra.txt" 2>&1 || { tail -30 "$O/extra.txt"; exit 1; }
      tail -25 "$O/extra.txt" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
find "$O" -name "*.csv" -size +2M -delete
echo done
