# full default bench (N = 1) on the current tree, then smoke
set -o pipefail
timeout -k 10 900 python -u bench.py > gpurun_out/r03u_bench.json 2> gpurun_out/r03u_bench.err || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03u_smoke.log 2>&1
