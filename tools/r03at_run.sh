# 11-bit onesweep digits for the bucket sort (rocPRIM config) vs hipCUB's default (8), and without rocPRIM's merge
# sort below 2^20 keys: parity, A/B at N = 1, solo G = 8
set -o pipefail
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03at_tests.log 2>&1 || exit $?
bash tools/ab_bench.sh r03at_ab tools/ab/lib_sort8.so tools/ab/lib_sortnm.so || exit $?
V="timeout -k 10 240 python -u tools/vrank_bench.py --solo --proofs 128 --steps 2 --cached --G 8"
for i in 1 2; do
  GPU_MAX_HW_QUEUES=32 $V | sed 's/}$/, "build": "default"}/' >> gpurun_out/r03at_solo.jsonl || exit $?
  SPX_LIB_PATH=tools/ab/lib_sort8.so GPU_MAX_HW_QUEUES=32 $V | sed 's/}$/, "build": "sort8"}/' >> gpurun_out/r03at_solo.jsonl || exit $?
  SPX_LIB_PATH=tools/ab/lib_sortnm.so GPU_MAX_HW_QUEUES=32 $V | sed 's/}$/, "build": "sortnm"}/' >> gpurun_out/r03at_solo.jsonl || exit $?
done
