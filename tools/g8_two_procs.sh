# Is one G = 8 rank process the limit, or the GPU? Two solo-rank processes side by side on one GPU
# (each half the proofs in flight and half the hardware queues; their timed regions aligned by a
# file barrier after the warm-up, tools/vrank_bench.py --sync-dir), against one process alone.
#   tools/g8_two_procs.sh TAG   -> gpurun_out/TAG.jsonl
set -e
TAG="$1"
O=gpurun_out/$TAG.jsonl
: > $O
one() {  # $1 label, $2 inflight, $3 queues, $4 sync dir, $5 sync n
  GPU_MAX_HW_QUEUES=$3 SPX_BLOCKING_SYNC=1 timeout -k 10 300 python tools/vrank_bench.py --G 8 --solo --inflight $2 \
    --proofs 64 --steps 10 --warmup 1 --sync-dir "$4" --sync-n $5 \
    | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); d['label']='$1'; print(json.dumps(d))"
}
for i in 1 2; do
  D=/tmp/g8sync_$i
  rm -rf $D /tmp/g8sync1_$i
  one single 64 32 /tmp/g8sync1_$i 1 >> $O
  ( one pairA 32 16 $D 2 > /tmp/pa.json ) & PA=$!
  ( one pairB 32 16 $D 2 > /tmp/pb.json ) & PB=$!
  wait $PA; wait $PB
  cat /tmp/pa.json /tmp/pb.json >> $O
done
