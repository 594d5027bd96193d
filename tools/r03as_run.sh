# kernel-trace concurrency of the solo G = 8 rank at the G >= 4 settings (64 in flight, 32 queues, level 0 batched)
set -eo pipefail
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/g8 -o run --output-format csv -- \
   python3 $R/tools/vrank_bench.py --G 8 --cached --solo --proofs 128 --steps 2 >> $R/gpurun_out/r03as.jsonl 2>> $R/gpurun_out/r03as.err
f=$(find /tmp/g8 -name "*kernel_trace.csv" | head -1)
TRACE_AFTER=k_sc1 TRACE_TOP=25 python3 $R/tools/trace_busy.py $f > $R/gpurun_out/r03as_busy_G8_inflight64.txt
find /tmp/g8 -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r03as_kernel_stats_G8_inflight64.csv \;
