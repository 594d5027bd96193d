# GPU suite from the RCCL tests on (the earlier files passed in r03v), then a short bench (no CPU baselines)
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_sharded.py tests/test_gpu_verify.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03x_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --no-cpu --steps 5 > gpurun_out/r03x_bench.json 2> gpurun_out/r03x_bench.err
