set -e
SPX_AB_SHARD_TAIL=3 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sharded.py tests/test_c2.py > gpurun_out/r05zu_test3.log 2>&1
SPX_AB_SHARD_TAIL=5 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sharded.py > gpurun_out/r05zu_test5.log 2>&1
VRANK_PROOFS=128 bash tools/ab_vrank.sh r05zu_ab_shardtail_G8 8 "SPX_AB_SHARD_TAIL=3" "SPX_AB_SHARD_TAIL=5"
