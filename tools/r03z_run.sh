# Fr add/sub carry chains + loads-first folds: parity of the Fr kernels, then A/B against the previous
# build and the non-temporal-store variant
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_c2.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03z_tests.log 2>&1 || exit $?
bash tools/ab_bench.sh r03z_ab tools/ab/lib_base.so tools/ab/lib_nt.so
