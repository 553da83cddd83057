#!/bin/bash
# One parameterised GPU-box runner (replaces the per-call scratch scripts of round 1).
#
#   gpurun --timeout 900 -- bash tools/gpurun.sh TAG STEP [STEP ...]
#
# Every step runs under its own time limit, logs to gpurun_out/TAG/, and the first failing step ends
# the call (no GPU work after a fault, abort or timeout).  Steps:
#   tests[:KEXPR]            pytest -m gpu [-k KEXPR] (default: all GPU tests)
#   smoke                    __graft_entry__.smoke()
#   bench[:BENCH_ARGS]       python bench.py BENCH_ARGS        (prints the JSON line)
#   prof[:BENCH_ARGS]        rocprofv3 --kernel-trace --stats of bench.py -> summary.txt (per step, warmup incl.)
#   pmc:COUNTERS[:CMD]       rocprofv3 --pmc COUNTERS (one pass) of CMD (default: attention microbench)
#   py:SCRIPT[:ARGS]         python SCRIPT ARGS                (microbenches, tools/*.py)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  log=$OUT/$n-$kind.log
  echo "[gpurun.sh] step $n: $step" | tee -a "$OUT/steps.txt"
  case $kind in
    tests)
      kx=()
      [ -n "$arg" ] && kx=(-k "$arg")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "${kx[@]}" > "$log" 2>&1
      rc=$?; tail -3 "$log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1
      rc=$?; tail -2 "$log" ;;
    bench)
      timeout -k 10 600 python -u bench.py ${arg} > "$log" 2>&1
      rc=$?; tail -1 "$log" ;;
    prof)
      d=$OUT/prof$n
      mkdir -p "$d"
      barg=${arg:---steps 3 --warmup 2}
      st=20; wu=5
      [[ "$barg" =~ --steps\ ([0-9]+) ]] && st=${BASH_REMATCH[1]}
      [[ "$barg" =~ --warmup\ ([0-9]+) ]] && wu=${BASH_REMATCH[1]}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$d" -o run -- python bench.py $barg > "$log" 2>&1
      rc=$?
      if [ $rc -eq 0 ]; then
        db=$(find "$d" -name "*.db" | head -n 1)
        csv=$(find "$d" -name "*kernel_stats.csv" | head -n 1)
        python tools/prof_summary.py "${db:-$csv}" $((st + wu)) > "$d/summary.txt" && head -12 "$d/summary.txt"
        rc=$?
        [ -n "$db" ] && rm -f "$db"
      fi ;;
    pmc)
      counters=${arg%%:*}
      cmd="python tools/attn_bench.py"
      [[ "$arg" == *:* ]] && cmd=${arg#*:}
      d=$OUT/pmc$n
      mkdir -p "$d"
      timeout -s KILL 120 rocprofv3 --pmc ${counters//,/ } --kernel-trace -d "$d" -o run -- $cmd > "$log" 2>&1
      rc=$?; tail -2 "$log" ;;
    py)
      script=${arg%%:*}
      sargs=""
      [[ "$arg" == *:* ]] && sargs=${arg#*:}
      timeout -k 10 600 python -u $script $sargs > "$log" 2>&1
      rc=$?; tail -4 "$log" ;;
    *)
      echo "unknown step $kind"; rc=2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "[gpurun.sh] step $n ($kind) failed rc=$rc"
    grep -E "Error|error|assert|FAILED|passed|failed" "$log" | tail -30
    exit $rc
  fi
done
echo "[gpurun.sh] all $n steps ok"
