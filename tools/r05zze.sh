set -e
bash tools/gpu.sh r05zze "samegpu=4,--steps 5 --warmup 2"
bash tools/ab_c2_env.sh r05zze_c2_hash "SPX_HASH_THREADS=12" "SPX_HASH_THREADS=24"
