#!/bin/bash
# Lists the counters rocprofv3 offers on this GPU (gpurun_out/pmc_list.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1
echo "rc=$?"; wc -l gpurun_out/pmc_list.txt
