set -e
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_interactive.py > gpurun_out/r05zy_test.log 2>&1
VRANK_PROOFS=128 bash tools/ab_vrank.sh r05zy_ab_copies_G8 8 r1cs-spartan_amd/libspartan_hip_alt1.so
