# same-GPU proof-sharded rehearsals: hardware-queue and in-flight variants (one GPU, N ranks)
set -o pipefail
run() {  # name, nproc, extra env / args
    local name=$1 np=$2; shift 2
    env SPX_BENCH_SAME_GPU=1 "$@" > gpurun_out/r03c_$name.json 2> gpurun_out/r03c_$name.err
}
P="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29512"
A="--steps 2 --warmup 1 --no-cpu --no-stats --no-cached --no-other"
run n4_hwq4 4 GPU_MAX_HW_QUEUES=4 timeout -k 10 300 $P --nproc-per-node 4 bench.py --gpus 4 $A || exit $?
run n4_inf4 4 timeout -k 10 300 $P --nproc-per-node 4 bench.py --gpus 4 $A --inflight 4 || exit $?
run n2 2 timeout -k 10 300 $P --nproc-per-node 2 bench.py --gpus 2 $A || exit $?
run n4_hwq4_inf4 4 GPU_MAX_HW_QUEUES=4 timeout -k 10 300 $P --nproc-per-node 4 bench.py --gpus 4 $A --inflight 4
