# ADVICE fixes (unwind drain, SPX_LVL0 agreement) on the GPU, then same-GPU N=2 / N=4 proof-sharded rehearsals
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiprocess.py tests/test_gpu_sharded.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ad_tests.log 2>&1 || exit $?
for N in 2 4; do
  SPX_BENCH_SAME_GPU=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus $N --steps 3 --warmup 1 --no-cpu --no-c2 --no-stats --rehearse '' --groups '' > gpurun_out/r03ad_rehearsal_n$N.json 2> gpurun_out/r03ad_rehearsal_n$N.err || exit $?
done
