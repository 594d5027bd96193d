# MSM tests + solo rehearsal G=1 traced + G=8 untraced
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread -k "msm or sharded or bit_exact_2_16" > gpurun_out/r03m_tests.log 2>&1 || exit $?
TRACE_GS=1 bash tools/r03j_run.sh || exit $?
timeout -k 10 200 python -u tools/vrank_bench.py --G 8 --inflight 16 --cached --solo --proofs 64 >> gpurun_out/r03m_solo.jsonl 2>> gpurun_out/r03m_solo.err
