# world = 8 code path on one GPU (8 processes time-sharing it): proof-sharded headline, batch mode and proof
# groups of 2, few contexts per rank (--inflight 4) to bound memory; then same-GPU N = 4 with proof groups
set -o pipefail
SPX_BENCH_SAME_GPU=1 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 8 --steps 1 --warmup 1 --no-cpu --no-c2 --no-stats --rehearse '' --inflight 4 --proofs-per-step 16 > gpurun_out/r03ap_n8.json 2> gpurun_out/r03ap_n8.err || exit $?
SPX_BENCH_SAME_GPU=1 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 \
    bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu --no-c2 --no-stats --rehearse '' > gpurun_out/r03ap_n4.json 2> gpurun_out/r03ap_n4.err
