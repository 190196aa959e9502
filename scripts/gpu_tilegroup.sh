#!/bin/bash
# Tile-group (GT x GJ) sweep of k_sweep_il: each prebuilt variant library is
# copied over libpdd.so in the box's scratch tree and the config-2 bench is run
# for f32 and u8.  Stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/tg; mkdir -p $O
for v in 8_4 4_4 16_4 8_8 8_2 16_2 4_8 16_8; do
  cp build/var/libpdd_$v.so pypulsar_amd/libpdd.so || exit 1
  for dt in f32 u8; do
    timeout -k 10 120 python bench.py --dtype $dt --steps 5 --warmup 2 --no-cpu-baseline > $O/$v.$dt.json 2> $O/$v.$dt.err || exit 2
    python -c "import json,sys;d=json.load(open('$O/$v.$dt.json'));print('$v','$dt',round(d['ms_per_step'],2),round(d['roofline']['kernel_ms'],2))" | tee -a $O/summary.txt
  done
done
