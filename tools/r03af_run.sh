# latency anatomy of one proof alone: solo rank of G = 1 and G = 8 (cached transcript), kernel trace
set -eo pipefail
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
for G in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/lat_$G -o run --output-format csv -- \
     python3 $R/tools/vrank_bench.py --G $G --inflight 1 --cached --solo --proofs 8 --steps 1 >> $R/gpurun_out/r03af.jsonl 2>> $R/gpurun_out/r03af.err
  f=$(find /tmp/lat_$G -name "*kernel_trace.csv" | head -1)
  cp $f $R/gpurun_out/r03af_trace_G$G.csv
  TRACE_AFTER=k_sc1_round TRACE_TOP=40 python3 $R/tools/trace_busy.py $f > $R/gpurun_out/r03af_busy_G$G.txt
done
