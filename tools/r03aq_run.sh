# (1) world = 8 code path on one GPU (r03ap); (2) weighting leaf of 2 buckets (SPX_TREE_CHUNK_LOG=1 build) vs 4, solo G = 8 and G = 1
set -o pipefail
bash tools/r03ap_run.sh || exit $?
V="timeout -k 10 240 python -u tools/vrank_bench.py --solo --proofs 128 --steps 2 --cached"
for i in 1 2; do
  GPU_MAX_HW_QUEUES=32 $V --G 8 | sed 's/}$/, "build": "default"}/' >> gpurun_out/r03aq.jsonl || exit $?
  SPX_LIB_PATH=tools/ab/lib_chunk1.so GPU_MAX_HW_QUEUES=32 $V --G 8 | sed 's/}$/, "build": "chunk1"}/' >> gpurun_out/r03aq.jsonl || exit $?
  GPU_MAX_HW_QUEUES=16 $V --G 1 | sed 's/}$/, "build": "default"}/' >> gpurun_out/r03aq.jsonl || exit $?
  SPX_LIB_PATH=tools/ab/lib_chunk1.so GPU_MAX_HW_QUEUES=16 $V --G 1 | sed 's/}$/, "build": "chunk1"}/' >> gpurun_out/r03aq.jsonl || exit $?
done
