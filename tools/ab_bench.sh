# A/B of two library builds on one box: $1 = alternative .so (SPX_LIB_PATH), default build second.
set -e
ALT="$1"; TAG="${2:-ab}"
for i in 1 2; do
  SPX_LIB_PATH="$ALT" timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${TAG}_alt_$i.json 2>/dev/null
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${TAG}_cur_$i.json 2>/dev/null
done
