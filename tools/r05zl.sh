set -e
export SPX_BLOCKING_SYNC=1 GPU_MAX_HW_QUEUES=4
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_group.py tests/test_c2.py > gpurun_out/r05zl_test.log 2>&1
O=gpurun_out/r05zl_c2group.jsonl
: > $O
for i in 1 2; do
  for cfg in "128 8" "64 8" "256 8" "192 8"; do
    set -- $cfg
    timeout -k 10 120 python tools/c2_cached.py --steps 16 --inflight $1 --group $2 >> $O
  done
done
