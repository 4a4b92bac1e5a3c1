set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tests/cpp/build/decision_test gpu > gpurun_out/decision_test.log 2>&1; rc=$?
tail -40 gpurun_out/decision_test.log; exit $rc
