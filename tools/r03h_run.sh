# solo-rank rehearsals: rank 0 of G with the GPU to itself (per-GPU work of an N = G node), cached transcript
set -o pipefail
for cfg in "1 16" "2 16" "4 16" "8 16" "8 32"; do
  set -- $cfg
  timeout -k 10 200 python -u tools/vrank_bench.py --G $1 --inflight $2 --cached --solo --proofs 64 >> gpurun_out/r03h_solo.jsonl 2>> gpurun_out/r03h_solo.err || exit $?
done
