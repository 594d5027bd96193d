# solo-rank G = 8, matrices absorbed per proof (the bench's rehearsal mode) vs index-cached, 64 / 32 in flight,
# hashing pool sizes (SPX_HASH_THREADS; default = one per context)
set -o pipefail
export GPU_MAX_HW_QUEUES=32 SPX_LVL0=batch
V="timeout -k 10 240 python -u tools/vrank_bench.py --G 8 --solo --proofs 128 --steps 2"
run() { # label, then args
  l=$1; shift
  env "$@" | sed "s/}\$/, \"cfg\": \"$l\"}/" >> gpurun_out/r03am.jsonl
}
for i in 1 2; do
  run cached64 $V --inflight 64 --cached || exit $?
  run absorbed64 $V --inflight 64 || exit $?
  run absorbed64_hash8 SPX_HASH_THREADS=8 $V --inflight 64 || exit $?
  run absorbed64_hash4 SPX_HASH_THREADS=4 $V --inflight 64 || exit $?
  run absorbed32 $V --inflight 32 || exit $?
done
