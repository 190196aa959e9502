#!/bin/bash
# Tile-group shapes of k_sweep_il (dev builds build/libpdd_<name>.so made by
# scripts/build_variant.sh <name> -DPDD_IL_GT=.. -DPDD_IL_GJ=..): per library,
# the configs[3] bench (HIP-event kernel time) and one rocprofv3 FETCH_SIZE
# pass of the same command.  LIBS: names.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/tile
mkdir -p $O
A="--config config3 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e"
for lib in ${LIBS:-base}; do
  PDD_DEV_LIB=build/libpdd_$lib.so timeout -k 10 300 python bench.py $A > $O/b_$lib.json 2> $O/b_$lib.err || { echo "bench $lib failed"; tail -3 $O/b_$lib.err; exit 1; }
  echo "$lib $(python -c "import json;d=json.load(open('$O/b_$lib.json'))['roofline'];print(d['kernel_ms_per_launch'], d['launches_per_step'])")"
  PDD_DEV_LIB=build/libpdd_$lib.so timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fe_$lib -o p --output-format csv -- python bench.py $A > $O/fe_$lib.log 2>&1 || { echo "fetch $lib failed"; tail -3 $O/fe_$lib.log; exit 1; }
done
echo TILE_OK
