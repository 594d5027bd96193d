# spin-then-block stream syncs (SPX_SYNC_SPIN_US, default 40) vs blocking only: parity smoke, A/B at N = 1,
# solo-rank G = 8 both ways; then the profiles of HEAD (kernel traces, PMC FETCH / WRITE / SQ passes, C2 passes)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bit_exact" > gpurun_out/r03ai_tests.log 2>&1 || exit $?
bash tools/ab_bench.sh r03ai_ab SPX_SYNC_SPIN_US=0 || exit $?
for i in 1 2; do
  timeout -k 10 200 python -u tools/vrank_bench.py --G 8 --inflight 16 --cached --solo --proofs 64 --steps 2 >> gpurun_out/r03ai_solo.jsonl || exit $?
  SPX_SYNC_SPIN_US=0 timeout -k 10 200 python -u tools/vrank_bench.py --G 8 --inflight 16 --cached --solo --proofs 64 --steps 2 >> gpurun_out/r03ai_solo.jsonl || exit $?
done
bash tools/profile_gpu.sh r03ai
