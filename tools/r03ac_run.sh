# re-entry check of HEAD on a fresh box: full GPU suite, smoke, then the default bench (CPU baselines included)
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ac_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ac_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r03ac_bench.json 2> gpurun_out/r03ac_bench.err
