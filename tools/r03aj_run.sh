# solo-rank G = 8 knob sweep (16 in flight unless noted), two alternating rounds: baseline, 32 in flight on
# 32 hardware queues, level 0 inside the first opening batch, shorter accumulation runs (G2 32 / G1 32)
set -o pipefail
V="timeout -k 10 200 python -u tools/vrank_bench.py --G 8 --cached --solo --proofs 64 --steps 2"
for i in 1 2; do
  $V --inflight 16 | sed 's/}$/, "cfg": "base"}/' >> gpurun_out/r03aj.jsonl || exit $?
  GPU_MAX_HW_QUEUES=32 $V --inflight 32 | sed 's/}$/, "cfg": "inflight32_hwq32"}/' >> gpurun_out/r03aj.jsonl || exit $?
  SPX_LVL0=batch $V --inflight 16 | sed 's/}$/, "cfg": "lvl0_batch"}/' >> gpurun_out/r03aj.jsonl || exit $?
  SPX_KSEG1=32 $V --inflight 16 | sed 's/}$/, "cfg": "kseg32"}/' >> gpurun_out/r03aj.jsonl || exit $?
done
