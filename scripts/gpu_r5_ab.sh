#!/bin/bash
# Round-5 A/B on one MI355X: the working-tree library against a reference
# build (REF=build/libpdd_<ref>.so, loaded through PDD_DEV_LIB), bench lines
# of the configs in CONFS, optional LDS/issue PMC passes and the GPU suite.
#   O=gpurun_out/<dir> REF=build/libpdd_c1.so BENCH="name|bench args;..." PMC=1 TESTS=1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/ab5}
mkdir -p $O
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { echo BUILD_FAIL; tail -5 $O/build.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.log; exit 1; }
echo SMOKE_OK
IFS=';' read -ra L <<< "${BENCH:-c3|--config config3;ns|--config northstar}"
for item in "${L[@]}"; do
  c=${item%%|*}; a=${item#*|}
  for lib in new ${REF:+ref}; do
    args="$a --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-e2e"
    if [ $lib = ref ]; then
      PDD_DEV_LIB=$REF timeout -k 10 300 python bench.py $args > $O/b_${c}_$lib.json 2> $O/b_${c}_$lib.err || { echo "bench $c $lib failed"; tail -3 $O/b_${c}_$lib.err; exit 1; }
    else
      timeout -k 10 300 python bench.py $args > $O/b_${c}_$lib.json 2> $O/b_${c}_$lib.err || { echo "bench $c $lib failed"; tail -3 $O/b_${c}_$lib.err; exit 1; }
    fi
    python - $O/b_${c}_$lib.json $c $lib <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = l.get("roofline") or {}
print("%-6s %-4s value %.4g  step %.2f ms  kernel %.2f ms/launch x %s  frac %.3f  %s  DB %s" % (
    sys.argv[2], sys.argv[3], l["value"], l["ms_per_step"], r.get("kernel_ms_per_launch") or 0,
    r.get("launches_per_step"), r.get("frac") or 0, l["config"].get("method", "")[:40],
    (l["config"].get("plan") or {}).get("dms_per_block")))
PY
  done
done
if [ -n "$PMC" ]; then
  O=$O/pmc bash scripts/gpu_pmc_lds.sh > $O/pmc.txt 2>&1 || { echo PMC_FAIL; tail -5 $O/pmc.txt; exit 1; }
  echo PMC_OK
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest ${TFILES:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?
  tail -3 $O/pytest_gpu.log
  exit $rc
fi
