set -e
export SPX_BLOCKING_SYNC=1 GPU_MAX_HW_QUEUES=4
O=gpurun_out/r05zq_c2poll.jsonl
: > $O
for i in 1 2; do
  for p in 20 10 5 2 0 50; do
    timeout -k 10 120 python tools/c2_cached.py --steps 16 --inflight 128 --group 8 --poll $p >> $O
  done
done
