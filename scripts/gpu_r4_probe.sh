#!/bin/bash
# Round-4 stage-2 probes: per-wave stamps (dev build, PDD_SWEEP_DEBUG=4) of the
# factorised configs[3] / north-star tiles, the staging-form A/B (PDD_FX_STAGE)
# and the timing-only decomposition (devdma build).
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4probe; mkdir -p $O
for p in ${STAMPS:-"u8:3" "u8:11" "ns:3"}; do
  IFS=: read kind st <<< "$p"
  PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_DEBUG=4 PDD_FX_STAGE=$st timeout -k 10 120 python scripts/probes/il_stamps.py $kind > $O/stamps_${kind}_$st.txt 2>&1 || { echo "stamps $p failed"; tail -3 $O/stamps_${kind}_$st.txt; exit 1; }
  echo "stamps $p done"
done
if [ -n "$RUNS" ]; then RUNS="$RUNS" RUNT="${RUNT:-}" TF=tests/test_gpu_factor.py TK=factor bash scripts/gpu_fxstage.sh || exit 1; fi
if [ -n "$DBGS" ]; then LIBS=devdma DBGS="$DBGS" CFGS="${CFGS:-config3}" bash scripts/gpu_decomp.sh || exit 1; fi
# (the S1 probe of round 4 -- stage 1 with nontemporal stores, no gain,
# profiles/r4probe -- was removed with its kernel instance)
