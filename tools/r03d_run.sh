# in-process virtual-rank throughput (one GPU): G = 1, 2, 4 at equal total contexts, index-cached transcript
set -o pipefail
for cfg in "1 16" "2 8" "4 4" "4 16" "8 2"; do
  set -- $cfg
  timeout -k 10 200 python -u tools/vrank_bench.py --G $1 --inflight $2 --cached >> gpurun_out/r03d_vrank.jsonl 2>> gpurun_out/r03d_vrank.err || exit $?
done
