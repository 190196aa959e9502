#!/bin/bash
# SQ counter passes over the sweep kernel (one rocprofv3 --pmc pass each,
# never combined with tracing domains), summarised by scripts/pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/sq
mkdir -p $O
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM"
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
rc=0
for dt in ${DTYPES:-f32 u8}; do
  for p in 1 2; do
    eval C=\$P$p
    timeout -s KILL 90 rocprofv3 --pmc $C -d $O/${dt}_p$p -o p --output-format csv -- python bench.py $ARGS --dtype $dt > $O/${dt}_p$p.log 2>&1 || { rc=$?; echo "pass $dt $p failed rc=$rc"; tail -5 $O/${dt}_p$p.log; break 2; }
  done
done
python scripts/pmc_summary.py $O > $O/summary.txt 2>&1
cat $O/summary.txt
exit $rc
