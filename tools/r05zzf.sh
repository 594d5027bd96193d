set -e
for so in r1cs-spartan_amd/libspartan_hip_alt1.so; do
  SPX_LIB_PATH=$so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_sharded.py >> gpurun_out/r05zzf_test.log 2>&1
done
VRANK_PROOFS=128 bash tools/ab_vrank.sh r05zzf_ab_fuse256_G8 8 r1cs-spartan_amd/libspartan_hip_alt1.so
bash tools/ab_bench.sh r05zzf_ab_fuse256_N1 r1cs-spartan_amd/libspartan_hip_alt1.so
O=gpurun_out/r05zzf_ab_fuse256_c2.jsonl
: > $O
for i in 1 2; do
  for so in default r1cs-spartan_amd/libspartan_hip_alt1.so; do
    if [ "$so" = default ]; then unset SPX_LIB_PATH; else export SPX_LIB_PATH=$so; fi
    SPX_BLOCKING_SYNC=1 GPU_MAX_HW_QUEUES=4 timeout -k 10 120 python tools/c2_cached.py --steps 16 --inflight 128 --group 8 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); d['build']='$so'; print(json.dumps(d))" >> $O
  done
done
