# wave-transposed opening folds (k_open_fold_wave) + the rank share's two products side by side in k_tree_top:
# parity (every proof, sharded, verifier), A/B against the sumcheck-waves-only build and the per-lane build,
# then solo-rank G = 8 rehearsals of both builds (the share matters only at G > 1)
set -o pipefail
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_c2.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py tests/test_gpu_verify.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ah_tests.log 2>&1 || exit $?
bash tools/ab_bench.sh r03ah_ab tools/ab/lib_sc.so tools/ab/lib_base.so || exit $?
for i in 1 2; do
  timeout -k 10 200 python -u tools/vrank_bench.py --G 8 --inflight 16 --cached --solo --proofs 64 --steps 2 >> gpurun_out/r03ah_solo.jsonl || exit $?
  SPX_LIB_PATH=tools/ab/lib_sc.so timeout -k 10 200 python -u tools/vrank_bench.py --G 8 --inflight 16 --cached --solo --proofs 64 --steps 2 >> gpurun_out/r03ah_solo.jsonl || exit $?
done
