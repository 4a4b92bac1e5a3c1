#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/rss_probe.py > gpurun_out/rss.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/rss.log; exit $rc
