# BASELINE C2 index-cached with lockstep groups: proofs in flight x group size x hardware queues
set -e
export SPX_BLOCKING_SYNC=1
O=gpurun_out/r05zi_c2group.jsonl
: > $O
for i in 1 2; do
  for cfg in "64 4 4" "64 8 4" "128 8 4" "96 8 4" "64 8 8" "128 8 8" "64 4 8"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$3 timeout -k 10 120 python tools/c2_cached.py --steps 8 --inflight $1 --group $2 >> $O
  done
done
