#!/bin/bash
# A/B of the short-grid tilings (configs[2] grouped sweeps): subband bench
# lines and kernel stats per tuning build (scripts/build_variant.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/r6sh}
mkdir -p $O
for v in ${VARIANTS:-b0 s8f7 s8f7d}; do
  PDD_DEV_LIB=build/libpdd_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_grouped.py tests/test_gpu_configs.py tests/test_gpu_parity.py -q -x -k "config2 or grouped or ddplan or subband or ds" --timeout 240 --timeout-method thread > $O/test_$v.log 2>&1 || { echo "TEST FAIL $v"; tail -20 $O/test_$v.log; exit 1; }
  echo "$v tests: $(tail -1 $O/test_$v.log)"
  for r in 1 2; do
    PDD_DEV_LIB=build/libpdd_$v.so timeout -k 10 300 python bench.py --config subband --no-cpu-baseline > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { echo "BENCH FAIL $v"; tail -5 $O/bench_${v}_$r.err; exit 1; }
    python - $O/bench_${v}_$r.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
st = d["roofline"]["stages"]
print(sys.argv[2], "step %.3f ms" % d["ms_per_step"], " ".join("%.3f" % s["ms"] for s in st),
      " ".join(str(s.get("tile_trials")) for s in st))
PY
  done
done
