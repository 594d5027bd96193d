# A/B in one call: solo G=8 rehearsal, default vs SPX_SEG1_FIT=0 (fixed 64 references per element), alternating
set -o pipefail
for r in 1 2 3; do
  for v in 1 0; do
    SPX_SEG1_FIT=$v timeout -k 10 200 python -u tools/vrank_bench.py --G 8 --inflight 16 --solo --proofs 64 --steps 5 --cached | sed "s/}$/, \"seg1_fit\": $v}/" >> gpurun_out/r03p_ab.jsonl 2>> gpurun_out/r03p_ab.err || exit $?
  done
done
