#!/bin/bash
# One parameterised GPU session (replaces the round-2 run_r2*.sh /
# profile_r2*.sh one-offs): run named steps in order on the MI355X box, each
# under its own time limit, stopping at the first failure; every output lands
# under OUTDIR (a gpurun_out/ path, merged back by gpurun).
#
#   tools/gpu_steps.sh OUTDIR STEP [STEP ...]
#
# STEP (fields split on the first two ':'):
#   tests[:K]              python -m pytest tests -m gpu [-k K]     -> tests.log
#   smoke                  __graft_entry__.smoke()                  -> smoke.log
#   bench:NAME[:ARGS]      python3 bench.py ARGS                    -> NAME.json
#   ab:NAME:LIB|ARGS       bench.py ARGS with SCREENFIT_LIB=LIB     -> NAME.json
#   trace:NAME[:ARGS]      rocprofv3 --kernel-trace --stats of bench.py ARGS
#                                                                   -> NAME/
#   pmc:NAME:SETS|ARGS     tools/pmc_passes.sh (one rocprofv3 --pmc run per
#                          counter set, SETS space-separated)      -> NAME/
#   cmd:NAME:COMMAND       any command (probe binaries)            -> NAME.txt
#
# e.g. tools/gpu_steps.sh gpurun_out/r3c tests \
#        "bench:gain_c3:--screen gain --workload config3 --no-fits --no-cpu-baseline"
set -o pipefail
out=$1
shift
mkdir -p "$out"
export TMPDIR=/tmp
# the library every step of this session loads (ab: steps name their own)
python3 -c "import sys, json; sys.path.insert(0, 'ska-sdp-screen-fitting_amd'); \
from ska_sdp_screen_fitting_amd._lib import library_identity; \
print(json.dumps(library_identity()))" > "$out/library.json" 
T_TEST=${T_TEST:-400}
T_BENCH=${T_BENCH:-300}
for step in "$@"; do
  kind=${step%%:*}
  rest=${step#*:}
  [ "$rest" = "$step" ] && rest=""
  name=${rest%%:*}
  args=${rest#*:}
  [ "$args" = "$rest" ] && args=""
  case $kind in
    tests)
      k=()
      [ -n "$name" ] && k=(-k "$name")
      timeout -k 10 "$T_TEST" python -u -m pytest tests -m gpu -x -q --timeout 200 \
        --timeout-method thread "${k[@]}" > "$out/tests.log" 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" \
        > "$out/smoke.log" 2>&1 ;;
    bench)
      timeout -k 10 "$T_BENCH" python3 -u bench.py $args > "$out/$name.json" \
        2> "$out/$name.err" ;;
    ab)
      lib=${args%%|*}
      bargs=${args#*|}
      SCREENFIT_LIB=$lib timeout -k 10 "$T_BENCH" python3 -u bench.py $bargs \
        > "$out/$name.json" 2> "$out/$name.err" ;;
    trace)
      mkdir -p "$out/$name"
      timeout -k 10 "$T_BENCH" rocprofv3 --kernel-trace --stats -f csv -d "$out/$name" \
        -o t -- python3 bench.py $args > "$out/$name/bench.json" 2> "$out/$name.err" ;;
    pmc)
      sets=${args%%|*}
      bargs=${args#*|}
      tools/pmc_passes.sh "$out/$name" "$sets" -- python3 bench.py $bargs ;;
    cmd)
      timeout -k 10 "$T_BENCH" bash -c "$args" > "$out/$name.txt" 2>&1 ;;
    *)
      echo "unknown step $step" >&2
      exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc"
  if [ $rc -ne 0 ]; then
    echo "stopping after failed step: $step" >&2
    exit $rc
  fi
done
echo ALL DONE
