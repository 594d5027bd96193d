# solo rehearsal: proofs in flight per rank at G = 2, 4, 8 (5 continuous steps of 64 proofs, per-proof absorbed)
set -o pipefail
for cfg in "8 16" "8 32" "8 64" "4 16" "4 32" "2 16" "2 32" "1 16" "1 32"; do
  set -- $cfg
  timeout -k 10 200 python -u tools/vrank_bench.py --G $1 --inflight $2 --solo --proofs 64 --steps 5 >> gpurun_out/r03q_solo.jsonl 2>> gpurun_out/r03q_solo.err || exit $?
done
