# wave-transposed sumcheck rounds (k_sc1_wave, k_sc2_wave): parity, A/B against the fold-rounds-only build and the
# per-lane build, then the one-proof latency anatomy (r03af)
set -o pipefail
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_c2.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ag_tests.log 2>&1 || exit $?
bash tools/ab_bench.sh r03ag_ab tools/ab/lib_fold.so tools/ab/lib_base.so || exit $?
bash tools/r03af_run.sh
