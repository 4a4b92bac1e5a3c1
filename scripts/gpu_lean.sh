# Lean BFS pass: parity with 4 lanes per node forced, then latency per batch size for G=1 / G=4
set -o pipefail
mkdir -p gpurun_out
OPENR_SPF_LEAN_G=4 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "grid or lvl or config or G100 or smoke or update or exact or multirank" > gpurun_out/g4_tests.log 2>&1; rc=$?; tail -2 gpurun_out/g4_tests.log; [ $rc -eq 0 ] || exit $rc
for gsel in 1 4; do
OPENR_SPF_LEAN_G=$gsel timeout -k 10 200 python -u scripts/batch_latency.py --sizes 640,1250,2500,5000,10000 > gpurun_out/batch_g$gsel.log 2>&1 || exit 1
echo "G=$gsel"; grep sources gpurun_out/batch_g$gsel.log | cut -c1-110
done
for n in 1250 10000; do
OPENR_SPF_BFS_PROF=1 timeout -k 10 120 python -u scripts/batch_latency.py --sizes $n --reps 3 > gpurun_out/prof_$n.log 2>&1 || exit 1
grep "bfs_ell:" gpurun_out/prof_$n.log | tail -1
done
