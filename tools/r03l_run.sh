# GPU tests (subset) + solo-rank rehearsals after the fence-free round reduction
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sharded or msm or bit_exact" > gpurun_out/r03l_tests.log 2>&1 || exit $?
for cfg in "1 16" "8 16"; do
  set -- $cfg
  timeout -k 10 200 python -u tools/vrank_bench.py --G $1 --inflight $2 --cached --solo --proofs 64 >> gpurun_out/r03l_solo.jsonl 2>> gpurun_out/r03l_solo.err || exit $?
done
