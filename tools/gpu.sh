#!/bin/bash
# One parameterised GPU-box recipe (run via gpurun from the repo root); replaces round 3's one-off
# tools/r03*_run.sh files.
#   tools/gpu.sh TAG STEP [STEP ...]
# STEP is one of
#   tests[=PYTEST_ARGS]   pytest -m gpu (default: the whole tests/ tree)           -> TAG_tests.log
#   smoke                 __graft_entry__.smoke()                                    -> TAG_smoke.log
#   bench[=ARGS]          python bench.py ARGS (default: the driver's no-flag run)   -> TAG_bench.json
#   samegpu=N[,ARGS]      bench.py --gpus N with every rank on GPU 0 (SPX_BENCH_SAME_GPU=1)
#                                                                                    -> TAG_samegpuN.json
#   profile               tools/profile_gpu.sh TAG (rocprofv3 traces + PMC passes)
#   ab=ALT1;ALT2...       tools/ab_bench.sh TAG ALT1 ALT2 ...
# Every step has its own time limit; the first failing step ends the script (no retries).
set -o pipefail
TAG="$1"; shift
O=gpurun_out
mkdir -p "$O"
for step in "$@"; do
  name="${step%%=*}"; arg=""
  [[ "$step" == *=* ]] && arg="${step#*=}"
  echo "[$TAG] step $step" >&2
  case "$name" in
    tests)
      # shellcheck disable=SC2086
      SPX_HEARTBEAT="$O/${TAG}_heartbeat.log" timeout -k 10 1100 python -u -m pytest ${arg:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$O/${TAG}_tests.log" 2>&1 || exit $? ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/${TAG}_smoke.log" 2>&1 || exit $? ;;
    bench)
      # shellcheck disable=SC2086
      timeout -k 10 900 python -u bench.py $arg > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err" || exit $? ;;
    samegpu)
      n="${arg%%,*}"; extra=""; [[ "$arg" == *,* ]] && extra="${arg#*,}"
      # shellcheck disable=SC2086
      SPX_BENCH_SAME_GPU=1 timeout -k 10 700 python -u bench.py --gpus "$n" $extra \
        > "$O/${TAG}_samegpu${n}.json" 2> "$O/${TAG}_samegpu${n}.err" || exit $? ;;
    profile)
      timeout -k 10 1100 bash tools/profile_gpu.sh "$TAG" || exit $? ;;
    ab)
      IFS=';' read -r -a alts <<< "$arg"
      timeout -k 10 1100 bash tools/ab_bench.sh "$TAG" "${alts[@]}" || exit $? ;;
    *)
      echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo "[$TAG] done" >&2
