# split-lane fold rounds (k_sc1_fold_quad, k_sc2_fold_pair): parity, then A/B against the single-lane build
set -o pipefail
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_c2.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ae_tests.log 2>&1 || exit $?
bash tools/ab_bench.sh r03ae_ab tools/ab/lib_base.so
