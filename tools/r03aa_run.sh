# flattened three-matrix loop in k_sparse3: parity (SpMV / eval_on_x incl. ragged and duplicate-column
# matrices, full proofs, virtual ranks), then A/B against the previous build
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_c2.py tests/test_gpu_sharded.py tests/test_gpu_verify.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03aa_tests.log 2>&1 || exit $?
bash tools/ab_bench.sh r03aa_ab tools/ab/lib_prev.so
