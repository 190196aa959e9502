#!/bin/bash
# The factorisation cost model's numbers (developer library, PDD_SWEEP_DEBUG
# bit 3) for the bench configs' plans.
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=${O:-gpurun_out/fxm}; mkdir -p $O
for a in "config2 --dtype u8" "config3" "northstar" "config2"; do
  n=$(echo $a | tr ' ' '_')
  PDD_SWEEP_DEBUG=8 PDD_DEV_LIB=build/libpdd_dbg.so timeout -k 10 300 python bench.py --config $a --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $O/$n.json 2> $O/$n.err || { echo "fail $a"; tail -3 $O/$n.err; exit 1; }
  echo "== $a"; grep fx_build $O/$n.err | sort -u
done
