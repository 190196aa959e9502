#!/bin/bash
# Several bench lines in one GPU call (no CPU baseline): prints config, plan
# variant/LDS, kernel ms per launch and T adds/s.  SETS: ';'-separated bench
# argument lists.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/set
SETS=${SETS:-"--config config3;--config config2;--config config2 --dtype u8;--config northstar"}
IFS=';' read -ra A <<< "$SETS"
i=0
for a in "${A[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $a --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/set/b$i.json 2> gpurun_out/set/b$i.err || { echo "FAIL: $a"; tail -5 gpurun_out/set/b$i.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/set/b$i.json'));r=d['roofline'];p=d['config']['plan']
print('%-36s value %.3g  ms/step %.1f  kernel %.1f ms x%d  %.2f T adds/s  variant %s lds %s' % ('$a', d['value'], d['ms_per_step'], r['kernel_ms_per_launch'], r['launches_per_step'], r['achieved'], p['variant'], p['lds_bytes']))"
done
