# kernel traces of solo-rank throughput runs (16 in flight): SIMD-time per kernel family at G = 1 and G = 8
set -eo pipefail
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
for G in ${TRACE_GS:-1 8}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/sj_$G -o run --output-format csv -- \
     python3 $R/tools/vrank_bench.py --G $G --inflight 16 --cached --solo --proofs 64 --warmup 1 >> $R/gpurun_out/r03j_solo.jsonl 2>> $R/gpurun_out/r03j_solo.err
  f=$(find /tmp/sj_$G -name "*kernel_trace.csv" | head -1)
  TRACE_AFTER=k_sc1_round TRACE_TOP=45 python3 $R/tools/trace_busy.py $f > $R/gpurun_out/r03j_busy_solo_G$G.txt
done
