# kernel-trace statistics of in-process virtual-rank runs (G = 1 and G = 4, 16 contexts, cached transcript)
set -eo pipefail
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
for cfg in "1 16" "2 8"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/vr_$1 -o run --output-format csv -- \
     python3 $R/tools/vrank_bench.py --G $1 --inflight $2 --cached --proofs 32 >> $R/gpurun_out/r03e_vrank.jsonl 2>> $R/gpurun_out/r03e_vrank.err
  find /tmp/vr_$1 -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r03e_kernel_stats_G$1.csv \;
  f=$(find /tmp/vr_$1 -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_busy.py $f > $R/gpurun_out/r03e_busy_G$1.txt
done
