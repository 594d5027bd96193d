# group tests + C2 bench with lockstep groups (config c2 alone), then the default bench line
set -e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_group.py tests/test_c2.py > gpurun_out/r05zj_test.log 2>&1
timeout -k 10 600 python bench.py --config c2 --steps 20 --warmup 2 --rehearse= > gpurun_out/r05zj_c2.json 2> gpurun_out/r05zj_c2.err
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/r05zj_bench.json 2> gpurun_out/r05zj_bench.err
