# solo rehearsal, 5 continuous steps of 64 proofs (as bench.py times them), G = 1, 2, 4, 8, per-proof absorbed and cached
set -o pipefail
for cfg in "1 16" "2 16" "4 16" "8 16" "8 32"; do
  set -- $cfg
  timeout -k 10 200 python -u tools/vrank_bench.py --G $1 --inflight $2 --solo --proofs 64 --steps 5 >> gpurun_out/r03o_solo.jsonl 2>> gpurun_out/r03o_solo.err || exit $?
  timeout -k 10 200 python -u tools/vrank_bench.py --G $1 --inflight $2 --solo --proofs 64 --steps 5 --cached >> gpurun_out/r03o_solo.jsonl 2>> gpurun_out/r03o_solo.err || exit $?
done
