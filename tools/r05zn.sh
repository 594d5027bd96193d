set -e
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config c2 --steps 20 --warmup 2 --rehearse= > gpurun_out/r05zn_c2.json 2> gpurun_out/r05zn_c2.err
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/r05zn_bench.json 2> gpurun_out/r05zn_bench.err
