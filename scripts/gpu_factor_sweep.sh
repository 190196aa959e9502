#!/bin/bash
# bench.py step time under each --factor choice for the configs given
#   CASES="stream|auto force2 force4 off;config2|auto force4" O=gpurun_out/<dir>
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=${O:-gpurun_out/facs}; mkdir -p $O
IFS=';' read -ra L <<< "$CASES"
for item in "${L[@]}"; do
  c=${item%%|*}
  for f in ${item#*|}; do
    n=${c// /_}_$f
    timeout -k 10 300 python bench.py --config $c --factor $f --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/$n.json 2> $O/$n.err || { echo "fail $c $f"; tail -3 $O/$n.err; continue; }
    python -c "
import json
d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
r=d['roofline']; print('%-22s %-7s %8.2f ms/step  %s %.2f ms  %s' % ('$c', '$f', d['ms_per_step'], r.get('kernel'), r.get('kernel_ms_per_launch', 0), d['config'].get('method', '')[:50]))"
  done
done
