# per-G proofs in flight / level-0 mode / 32 hardware queues: sharded tests, the default bench (rehearsals at the new
# settings), A/B of 32 vs 16 hardware queues at N = 1, same-GPU N = 2 / 4 rehearsals
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_multiprocess.py tests/test_abi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03al_tests.log 2>&1 || exit $?
timeout -k 10 700 python -u bench.py > gpurun_out/r03al_bench.json 2> gpurun_out/r03al_bench.err || exit $?
bash tools/ab_bench.sh r03al_ab GPU_MAX_HW_QUEUES=16 || exit $?
for N in 2 4; do
  SPX_BENCH_SAME_GPU=1 timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus $N --steps 3 --warmup 1 --no-cpu --no-c2 --no-stats --rehearse '' --groups '' > gpurun_out/r03al_rehearsal_n$N.json 2> gpurun_out/r03al_rehearsal_n$N.err || exit $?
done
