# sharded GPU tests + virtual-rank throughput after the round-robin bucket assignment
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_multiprocess.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03g_tests.log 2>&1 || exit $?
for cfg in "1 16" "2 8" "4 4" "8 2"; do
  set -- $cfg
  timeout -k 10 200 python -u tools/vrank_bench.py --G $1 --inflight $2 --cached >> gpurun_out/r03g_vrank.jsonl 2>> gpurun_out/r03g_vrank.err || exit $?
done
