# counting sort vs radix sort: correctness (MSM + sharded tests) and A/B of solo rehearsals at G = 1, 8
set -o pipefail
SPX_MSM_SORT=count timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread -k "msm or sharded or bit_exact" > gpurun_out/r03t_tests.log 2>&1 || exit $?
for r in 1 2; do
  for G in 1 8; do
    for v in radix count; do
      SPX_MSM_SORT=$v timeout -k 10 200 python -u tools/vrank_bench.py --G $G --inflight 16 --solo --proofs 64 --steps 3 --cached | sed "s/}$/, \"sort\": \"$v\"}/" >> gpurun_out/r03t_ab.jsonl 2>> gpurun_out/r03t_ab.err || exit $?
    done
  done
done
