#!/bin/bash
# Timing decomposition of the sweep kernel with the dev build:
# PDD_SWEEP_DEBUG=0 full, =1 no staging DMAs, =2 no MFMA compute, =3 neither.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/dbg
for dbg in ${DBGS:-0 1 2 3}; do
  PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_MX=${MX:-1} PDD_SWEEP_DEBUG=$dbg timeout -k 10 200 python bench.py ${BENCHX:---steps 3 --warmup 1} --no-cpu-baseline > gpurun_out/dbg/b$dbg.json 2> gpurun_out/dbg/b$dbg.err || { tail -5 gpurun_out/dbg/b$dbg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/dbg/b$dbg.json'));r=d['roofline'];print('dbg $dbg', 'ms/launch %.1f' % r['kernel_ms_per_launch'], 'T %.2f' % r['achieved'], d['config']['plan'])"
done
