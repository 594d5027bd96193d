# proofs in flight x hardware queues x level-0 mode, solo-rank G = 1, 2, 4, 8 (index-cached transcript)
set -o pipefail
V="timeout -k 10 240 python -u tools/vrank_bench.py --cached --solo --proofs 128 --steps 1"
run() {  # G inflight hwq lvl0
  GPU_MAX_HW_QUEUES=$3 SPX_LVL0=$4 $V --G $1 --inflight $2 | sed "s/}\$/, \"hwq\": $3, \"lvl0\": \"$4\"}/" >> gpurun_out/r03ak.jsonl
}
for i in 1 2; do
  run 8 32 32 side || exit $?
  run 8 32 32 batch || exit $?
  run 8 64 32 batch || exit $?
  run 1 16 16 side || exit $?
  run 1 32 32 side || exit $?
  run 1 32 32 batch || exit $?
done
for G in 2 4; do
  run $G 16 16 side || exit $?
  run $G 32 32 batch || exit $?
done
