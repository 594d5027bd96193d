set -e
export SPX_BLOCKING_SYNC=1 GPU_MAX_HW_QUEUES=4
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_group.py > gpurun_out/r05zh_test.log 2>&1
O=gpurun_out/r05zh_c2group.jsonl
: > $O
for i in 1 2; do
  for g in 1 2 4 8; do
    timeout -k 10 120 python tools/c2_cached.py --steps 8 --inflight 32 --group $g >> $O
  done
  timeout -k 10 120 python tools/c2_cached.py --steps 8 --inflight 64 --group 8 >> $O
done
