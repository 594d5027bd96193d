# sumcheck-1 messages by finite differences (host): parity (every proof byte), C2, sharded; then the default bench of HEAD
set -o pipefail
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_c2.py tests/test_gpu_sharded.py tests/test_gpu_verify.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03au_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/r03au_bench.json 2> gpurun_out/r03au_bench.err
