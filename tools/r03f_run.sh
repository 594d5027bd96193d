# virtual-rank throughput vs hardware queues (one GPU, cached transcript)
set -o pipefail
for cfg in "1 16 16" "1 16 32" "4 4 16" "4 4 32" "4 4 8" "2 8 32"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$3 timeout -k 10 200 python -u tools/vrank_bench.py --G $1 --inflight $2 --cached | sed "s/}$/, \"hwq\": $3}/" >> gpurun_out/r03f_vrank.jsonl 2>> gpurun_out/r03f_vrank.err || exit $?
done
