# A/B (one box, alternating): solo rehearsals G = 1, 4, 8: default / level 0 inside the first opening /
# 32 hardware queues + 32 in flight (5 continuous steps of 64 proofs, per-proof absorbed, as bench.py)
set -o pipefail
v() { timeout -k 10 200 env "$@" | sed "s/}$/, \"cfg\": \"$CFG\"}/" >> gpurun_out/r03w_ab.jsonl 2>> gpurun_out/r03w_ab.err; }
for r in 1 2; do
  for G in 1 4 8; do
    CFG=default v python -u tools/vrank_bench.py --G $G --inflight 16 --solo --proofs 64 --steps 5 || exit $?
    CFG=lvl0batch v SPX_LVL0=batch python -u tools/vrank_bench.py --G $G --inflight 16 --solo --proofs 64 --steps 5 || exit $?
    CFG=hwq32 v GPU_MAX_HW_QUEUES=32 python -u tools/vrank_bench.py --G $G --inflight 32 --solo --proofs 64 --steps 5 || exit $?
  done
done
