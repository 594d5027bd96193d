# Launch rate of one process against two side by side (tools/ubench_launch.hip): run via gpurun.
set -e
O=gpurun_out/$1.jsonl
: > $O
for q in 4 32; do
  for b in 1 4; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 tools/ubench_launch 64 2000 $b | sed "s/^{/{\"procs\": 1, \"hwq\": $q, /" >> $O
    ( GPU_MAX_HW_QUEUES=$((q / 2 > 0 ? q / 2 : 1)) timeout -k 10 120 tools/ubench_launch 32 2000 $b > /tmp/la.json ) & A=$!
    ( GPU_MAX_HW_QUEUES=$((q / 2 > 0 ? q / 2 : 1)) timeout -k 10 120 tools/ubench_launch 32 2000 $b > /tmp/lb.json ) & B=$!
    wait $A; wait $B
    sed "s/^{/{\"procs\": 2, \"hwq\": $q, \"half\": \"a\", /" /tmp/la.json >> $O
    sed "s/^{/{\"procs\": 2, \"hwq\": $q, \"half\": \"b\", /" /tmp/lb.json >> $O
  done
done
