set -e
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_c2.py tests/test_gpu_interactive.py tests/test_gpu_group.py > gpurun_out/r05zt_test.log 2>&1
bash tools/ab_env.sh r05zt_ab_hosttail1 "SPX_AB_HOST_TAIL1=0"
