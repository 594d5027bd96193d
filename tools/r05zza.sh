set -e
for so in r1cs-spartan_amd/libspartan_hip_alt1.so r1cs-spartan_amd/libspartan_hip_alt2.so; do
  SPX_LIB_PATH=$so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_sharded.py >> gpurun_out/r05zza_test.log 2>&1
done
VRANK_PROOFS=128 bash tools/ab_vrank.sh r05zza_ab_seg_chunk_G8 8 r1cs-spartan_amd/libspartan_hip_alt1.so r1cs-spartan_amd/libspartan_hip_alt2.so
bash tools/ab_bench.sh r05zza_ab_seg_chunk_N1 r1cs-spartan_amd/libspartan_hip_alt1.so r1cs-spartan_amd/libspartan_hip_alt2.so
