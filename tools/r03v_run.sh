# batch-affine microbenchmark, full GPU suite, then a short bench (no CPU baselines)
set -o pipefail
timeout -k 10 120 tools/ubench_batch_affine > gpurun_out/r03v_ubench_batch_affine.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03v_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --no-cpu --steps 5 > gpurun_out/r03v_bench.json 2> gpurun_out/r03v_bench.err
