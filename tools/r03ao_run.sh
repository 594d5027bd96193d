# BASELINE C4 shape: 2^22, solo-rank G = 8 (64 in flight, 32 queues) vs G = 1 (16 in flight, 16 queues), matrices absorbed per proof
set -o pipefail
timeout -k 10 500 env GPU_MAX_HW_QUEUES=16 python -u tools/vrank_bench.py --G 1 --solo --log-n 22 --proofs 64 --steps 1 >> gpurun_out/r03ao_c4.jsonl || exit $?
timeout -k 10 500 env GPU_MAX_HW_QUEUES=32 python -u tools/vrank_bench.py --G 8 --solo --log-n 22 --proofs 64 --steps 1 >> gpurun_out/r03ao_c4.jsonl || exit $?
timeout -k 10 500 env GPU_MAX_HW_QUEUES=32 python -u tools/vrank_bench.py --G 4 --solo --log-n 22 --proofs 64 --steps 1 >> gpurun_out/r03ao_c4.jsonl || exit $?
