#!/bin/bash
# The 8-rank configs[3] step rehearsed on one GPU: time split
# (resident + PCIe-inclusive legs) and DM split, one bench line each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/r6rh}
mkdir -p $O
for m in timeshard dmshard; do
  timeout -k 10 500 python bench.py --rehearse 8 --mode $m > $O/rehearse8_$m.json 2> $O/rehearse8_$m.err || { echo "FAIL $m"; tail -5 $O/rehearse8_$m.err; exit 1; }
  cut -c1-400 $O/rehearse8_$m.json
done
