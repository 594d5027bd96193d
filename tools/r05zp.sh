set -e
export SPX_BLOCKING_SYNC=1 GPU_MAX_HW_QUEUES=4
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_group.py tests/test_c2.py tests/test_gpu_parity.py > gpurun_out/r05zp_test.log 2>&1
O=gpurun_out/r05zp_ab_col.jsonl
: > $O
for i in 1 2 3; do
  for so in default r1cs-spartan_amd/libspartan_hip_alt1.so; do
    if [ "$so" = default ]; then unset SPX_LIB_PATH; else export SPX_LIB_PATH=$so; fi
    timeout -k 10 120 python tools/c2_cached.py --steps 16 --inflight 128 --group 8 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); d['build']='$so'; print(json.dumps(d))" >> $O
    timeout -k 10 120 python tools/c2_cached.py --steps 8 --inflight 32 --group 1 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); d['build']='$so'; print(json.dumps(d))" >> $O
  done
done
