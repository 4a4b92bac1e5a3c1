# Strong-scaling shard latency: wave pass (auto) vs the lean pass with delta rows.
set -o pipefail
mkdir -p gpurun_out
for w in 2 0; do
  OPENR_SPF_BFS_WAVE=$w timeout -k 10 200 python -u scripts/batch_latency.py --topology grid100 --sizes 1250,2500,3334,5000,10000 > gpurun_out/shards_$w.log 2>&1 || { tail -20 gpurun_out/shards_$w.log; exit 1; }
  echo "wave=$w"; grep '{' gpurun_out/shards_$w.log
done
