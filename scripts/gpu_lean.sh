set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 tests/cpp/build/decision_test gpu > gpurun_out/dec.log 2>&1 || { grep -E "FAIL|expected|Error|error" gpurun_out/dec.log | head -30; tail -5 gpurun_out/dec.log; exit 1; }
grep -E "FAIL|tests,|prefetch=|HostThreads|Ksp2Route" gpurun_out/dec.log
timeout -k 10 300 tests/cpp/build/linkstate_test gpu > gpurun_out/ls.log 2>&1 || { grep -E "FAIL" gpurun_out/ls.log | head; tail -5 gpurun_out/ls.log; exit 1; }
grep -E "FAIL|tests," gpurun_out/ls.log
