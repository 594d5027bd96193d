set -e
export SPX_BLOCKING_SYNC=1 GPU_MAX_HW_QUEUES=4
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_group.py tests/test_c2.py > gpurun_out/r05zs_test.log 2>&1
O=gpurun_out/r05zs_hosttail.jsonl
: > $O
for i in 1 2; do
  for h in 5 0 3 4; do
    SPX_AB_HOST_TAIL=$h timeout -k 10 120 python tools/c2_cached.py --steps 16 --inflight 128 --group 8 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); d['host_tail']=$h; print(json.dumps(d))" >> $O
  done
done
