# (r03ab) compacted keys with one digit pass; sharded parity first
# PMC pass (VALU instructions, waves, busy cycles) over solo-rank rehearsals G = 1 and G = 8, one proof in flight
set -eo pipefail
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
(cd $R && timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_multiprocess.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/r03ab_tests.log 2>&1)
for G in 1 8; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_BUSY_CYCLES -d /tmp/pv_$G -o run --output-format csv -- \
     python3 $R/tools/vrank_bench.py --G $G --inflight 1 --solo --proofs 4 --warmup 0 --cached >> $R/gpurun_out/r03ab_pmc.jsonl 2>> $R/gpurun_out/r03ab_pmc.err
  f=$(find /tmp/pv_$G -name "*counter_collection.csv" | head -1)
  cp $f $R/gpurun_out/r03ab_counters_G$G.csv; python3 $R/tools/valu_summary.py $f 4 > $R/gpurun_out/r03ab_valu_G$G.txt 2>&1 || true
done
