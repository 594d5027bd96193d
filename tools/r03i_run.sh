# kernel-trace statistics of a solo rank (one proof in flight): per-rank device work of G = 1 and G = 8
set -eo pipefail
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
for G in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/so_$G -o run --output-format csv -- \
     python3 $R/tools/vrank_bench.py --G $G --inflight 1 --cached --solo --proofs 8 --warmup 1 >> $R/gpurun_out/r03i_solo.jsonl 2>> $R/gpurun_out/r03i_solo.err
  find /tmp/so_$G -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r03i_kernel_stats_solo_G$G.csv \;
done
