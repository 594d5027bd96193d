set -o pipefail
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err || exit $?
SPX_BENCH_SAME_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu > gpurun_out/r03b_rehearsal_n4.json 2> gpurun_out/r03b_rehearsal_n4.err
