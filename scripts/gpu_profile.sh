#!/bin/bash
# rocprofv3 passes over the default bench (sweep kernel): kernel trace + stats,
# then separate PMC passes (never combined with tracing domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
ARGS=${BENCH_ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline"}
python -c "import __graft_entry__ as g; g.build()" || exit 1
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- python bench.py $ARGS > gpurun_out/prof_kt.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS -d gpurun_out/prof_pmc1 -o p1 --output-format csv -- python bench.py $ARGS > gpurun_out/prof_pmc1.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_pmc2 -o p2 --output-format csv -- python bench.py $ARGS > gpurun_out/prof_pmc2.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/prof_pmc3 -o p3 --output-format csv -- python bench.py $ARGS > gpurun_out/prof_pmc3.log 2>&1 \
 && echo PROFILE_OK
rc=$?
tail -3 gpurun_out/prof_*.log
find gpurun_out/prof_* -name "*.csv" | head -20
exit $rc
