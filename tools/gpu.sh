#!/bin/bash
# One parameterised GPU script for every diagnostic / evidence run (replaces
# the round-specific gpu_r0x*.sh one-offs).  Each STEP runs under its own time
# limit, writes gpurun_out/TAG/<step>.txt, prints its tail; the first failing
# step ends the call (nothing runs on the GPU after a fault or a timeout).
#
#   tools/gpu.sh TAG STEP [STEP ...]
#
# STEP:
#   pytest[=EXPR]          pytest -m gpu (optionally -k EXPR)
#   smoke                  __graft_entry__.smoke()
#   bench[=ARGS]           python bench.py ARGS (default: the driver's default line) -> bench.json
#   kbench=CONFIG          bench.py --config CONFIG --kernel-only --no-cpu -> bench_CONFIG.json
#   ablate=CONFIG:NFAM:LIBS  tools/ablate.py (LIBS comma-separated libdcr_*.so names), outputs checked
#   stamps=CONFIG:LIB      tools/stamps.py with a DCR_STAMP build
#   kt=ARGS                rocprofv3 --kernel-trace --stats over bench.py ARGS -> kt/, kernel_grid.csv
#   traffic                FETCH_SIZE / WRITE_SIZE passes over the C2 kernel bench -> traffic.json
#   pmc=COUNTERS:LIB       one rocprofv3 --pmc pass over tools/ablate.py on LIB (C2)
#   inflate=NMEM           tools/inflate_speed.py
#   dfl                    tools/deflate_probe.py
#   py=SCRIPT ARGS         any python script (quoted as one step)
#   env=NAME=VALUE         export a variable for the later steps (A/B knobs: DCR_SCAN_THREADS, ...)
set -o pipefail
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
O=gpurun_out/$TAG
L=duplexumiconsensusreads_amd
mkdir -p "$O"
run() {   # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$O/$name.txt" 2>&1
  local rc=$?
  tail -${TAILN:-15} "$O/$name.txt"
  echo "== $name rc=$rc"
  return $rc
}
for step in "$@"; do
  key=${step%%=*}; val=${step#*=}; [ "$val" = "$step" ] && val=""
  case $key in
    pytest)
      if [ -n "$val" ]; then run pytest 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$val" || exit 1
      else run pytest 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1; fi ;;
    smoke) run smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench)
      # shellcheck disable=SC2086
      run bench 600 python3 -u bench.py $val || exit 1
      grep '^{' "$O/bench.txt" | tail -1 > "$O/bench.json" ;;
    kbench)
      run "kbench_$val" 300 python3 -u bench.py --config "$val" --kernel-only --no-cpu || exit 1
      grep '^{' "$O/kbench_$val.txt" | tail -1 > "$O/bench_$val.json" ;;
    ablate)
      IFS=: read -r cfg nfam libs <<< "$val"
      paths=""; for l in ${libs//,/ }; do paths="$paths $PWD/$L/$l"; done
      # shellcheck disable=SC2086
      ABL_CONFIG=$cfg run "ablate_$cfg" 400 python3 -u tools/ablate.py "$nfam" $paths || exit 1 ;;
    stamps)
      IFS=: read -r cfg lib <<< "$val"
      ABL_CONFIG=$cfg run "stamps_$cfg" 300 python3 -u tools/stamps.py 312500 "$PWD/$L/$lib" || exit 1 ;;
    kt)
      k=$(( ${k:-0} + 1 )); sfx=$([ "$k" = 1 ] && echo "" || echo "$k")
      # shellcheck disable=SC2086
      run "kt$sfx" 600 rocprofv3 --kernel-trace --stats -d "$O/kt$sfx" -o kt --output-format csv -- python3 bench.py $val || exit 1
      find "$O/kt$sfx" -name "*kernel_trace.csv" -exec python3 tools/kt_grid.py {} \; > "$O/kernel_grid$sfx.csv" || exit 1
      find "$O/kt$sfx" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats$sfx.csv" \;
      grep '^{' "$O/kt$sfx.txt" | tail -1 > "$O/bench_kt$sfx.json" ;;
    traffic) run "traffic$val" 600 bash tools/gpu_traffic.sh "$TAG" $val || exit 1 ;;   # traffic=C3: that config
    pmc)
      IFS=: read -r ctrs lib <<< "$val"
      # shellcheck disable=SC2086
      n=$(( ${n:-0} + 1 )); run "pmc${n}_${lib%.so}" 120 rocprofv3 --pmc ${ctrs//,/ } -d "$O/pmc${n}_${lib%.so}" -o pmc -- python3 tools/ablate.py 312500 "$PWD/$L/$lib" || exit 1
      python3 tools/pmc_db.py "$O/pmc${n}_${lib%.so}" 1250000 k_consensus_fast k_fast_rows > "$O/pmc${n}_${lib%.so}.sum" && cat "$O/pmc${n}_${lib%.so}.sum" ;;
    inflate) run inflate 300 python3 -u tools/inflate_speed.py "${val:-100000}" 1 || exit 1 ;;
    dfl) run dfl 300 python3 -u tools/deflate_probe.py || exit 1 ;;
    env) export "${val?}"; echo "== env $val" ;;
    py)
      # shellcheck disable=SC2086
      run "py_$(basename "${val%% *}" .py)" 1100 python3 -u $val || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
