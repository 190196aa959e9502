#!/bin/bash
# Round-5 stage-2 probes (developer build build/libpdd_dev.so): per-wave
# stamps of the factorised configs[3] / north-star tiles, then the timing-only
# decomposition (PDD_SWEEP_DEBUG 0 production, 1 no window staging, 2 no
# reads/adds, 3 neither) of both configs' bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/probe5}
mkdir -p $O
for kind in u8 ns; do
  PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_DEBUG=4 timeout -k 10 180 python scripts/probes/il_stamps.py $kind > $O/stamps_$kind.txt 2>&1 || { echo "stamps $kind failed"; tail -3 $O/stamps_$kind.txt; exit 1; }
  head -4 $O/stamps_$kind.txt
done
for c in config3 northstar; do
  for dbg in 0 1 2 3; do
    PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_DEBUG=$dbg timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/b_${c}_$dbg.json 2> $O/b_${c}_$dbg.err || { echo "bench $c $dbg failed"; tail -3 $O/b_${c}_$dbg.err; exit 1; }
    echo "$c dbg=$dbg $(python -c "import json;d=json.loads(open('$O/b_${c}_$dbg.json').read().strip().splitlines()[-1])['roofline'];print('%.2f ms/launch x %s' % (d['kernel_ms_per_launch'], d['launches_per_step']))")"
  done
done
