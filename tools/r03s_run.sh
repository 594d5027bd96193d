# kernel-trace concurrency of solo G=8 rehearsals: 16 in flight / 16 hardware queues vs 32 / 32
set -eo pipefail
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
for cfg in "16 16" "32 32"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/sc_$1 -o run --output-format csv -- \
     python3 $R/tools/vrank_bench.py --G 8 --inflight $2 --cached --solo --proofs 64 --steps 3 >> $R/gpurun_out/r03s.jsonl 2>> $R/gpurun_out/r03s.err
  f=$(find /tmp/sc_$1 -name "*kernel_trace.csv" | head -1)
  TRACE_AFTER=k_sc1_round TRACE_TOP=25 python3 $R/tools/trace_busy.py $f > $R/gpurun_out/r03s_busy_hwq$1.txt
done
