# solo G=8 rehearsal vs hardware queues and proofs in flight (cached transcript)
set -o pipefail
for cfg in "16 16" "32 32" "32 16" "8 16" "16 48"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 python -u tools/vrank_bench.py --G 8 --inflight $2 --cached --solo --proofs 96 | sed "s/}$/, \"hwq\": $1}/" >> gpurun_out/r03n_solo.jsonl 2>> gpurun_out/r03n_solo.err || exit $?
done
