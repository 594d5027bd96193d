# GPU tests of the launch-lean MSM / sumcheck + solo-rank rehearsals
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "sharded or msm or commit_open or bit_exact or multiprocess or sum_over or eval_on" > gpurun_out/r03k_tests.log 2>&1 || exit $?
for cfg in "1 16" "2 16" "4 16" "8 16"; do
  set -- $cfg
  timeout -k 10 200 python -u tools/vrank_bench.py --G $1 --inflight $2 --cached --solo --proofs 64 >> gpurun_out/r03k_solo.jsonl 2>> gpurun_out/r03k_solo.err || exit $?
done
