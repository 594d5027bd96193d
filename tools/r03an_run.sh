# hashing pool sized to the core budget; default bench with child-process rehearsals; same-GPU N = 4
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_multiprocess.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03an_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/r03an_bench.json 2> gpurun_out/r03an_bench.err || exit $?
SPX_BENCH_SAME_GPU=1 timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 4 --steps 3 --warmup 1 --no-cpu --no-c2 --no-stats --rehearse '' --groups '' > gpurun_out/r03an_rehearsal_n4.json 2> gpurun_out/r03an_rehearsal_n4.err
