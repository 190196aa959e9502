#!/bin/bash
# Interleaved sweep variants: parity, kernel time, per-wave stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/il
mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
VARS=${VARS:-0 1 2 3 4}
VARS="$VARS" NOSQ=1 bash scripts/gpu_ws.sh || exit 1
timeout -k 10 300 python scripts/probes/il_stamps.py $VARS > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep "^v=" $O/stamps.log
