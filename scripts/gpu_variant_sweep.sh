#!/bin/bash
# Dev build: force each candidate tiling (PDD_SWEEP_VARIANT = first index tried)
# on a few bench configs; prints kernel ms per launch and the variant chosen.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/vs
for cfg in ${CFGS:-"config3:u8" "northstar:u8" "config2:u8" "config2:f32"}; do
  c=${cfg%%:*}; dt=${cfg##*:}
  for v in ${VARS:-0 1 2 3 4 5 6}; do
    PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_VARIANT=$v timeout -k 10 200 python bench.py --config $c --dtype $dt --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/vs/b.json 2> gpurun_out/vs/b.err || { echo "FAIL $c $dt $v"; tail -3 gpurun_out/vs/b.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/vs/b.json'));r=d['roofline'];p=d['config']['plan']
print('$c $dt force %s -> variant %s lds %6d kernel %.1f ms  %.2f T' % ('$v', p['variant'], p['lds_bytes'], r['kernel_ms_per_launch'], r['achieved']))"
  done
done
