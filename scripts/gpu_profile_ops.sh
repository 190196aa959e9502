#!/bin/bash
# rocprofv3 over `bench.py --config ops`: kernel trace + stats, then separate
# FETCH_SIZE / WRITE_SIZE passes (HBM-side bytes per single-DM kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
ARGS="--config ops --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ops_kt -o kt --output-format csv -- python bench.py $ARGS > gpurun_out/ops_kt.log 2>&1 \
 && timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/ops_pmc2 -o p2 --output-format csv -- python bench.py $ARGS > gpurun_out/ops_pmc2.log 2>&1 \
 && timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/ops_pmc3 -o p3 --output-format csv -- python bench.py $ARGS > gpurun_out/ops_pmc3.log 2>&1 \
 && echo PROFILE_OK
rc=$?
tail -2 gpurun_out/ops_*.log
exit $rc
