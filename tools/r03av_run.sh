# parity of HEAD (sumcheck-1 message stepping): every proof byte vs the oracle, sharded, C2; smoke
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_c2.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03av_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03av_smoke.log 2>&1
