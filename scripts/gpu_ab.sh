#!/bin/bash
# A/B timing of developer builds of libpdd (LIBS = names of build/libpdd_<name>.so)
# on a few bench configs; prints the sweep kernel ms per launch.  Then the
# sweep GPU tests on the build named by TESTLIB (if set).
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
for cfg in ${CFGS:-"config3:u8" "config2:u8" "config2:f32"}; do
  c=${cfg%%:*}; dt=${cfg##*:}
  for lib in ${LIBS:-base dev}; do
    PDD_DEV_LIB=build/libpdd_$lib.so timeout -k 10 200 python bench.py --config $c --dtype $dt --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-e2e ${BARGS} > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { echo "FAIL $c $dt $lib"; tail -3 gpurun_out/ab/b.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/ab/b.json'));r=d['roofline'];p=d['config']['plan']
print('$c $dt %-6s variant %s kernel %.2f ms  %.2f T  step %.1f ms' % ('$lib', p['variant'], r['kernel_ms_per_launch'], r['achieved'], d['ms_per_step']))"
  done
done
if [ -n "$TESTLIB" ]; then
  PDD_DEV_LIB=build/libpdd_$TESTLIB.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/ab/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/ab/pytest.log; exit $rc
fi
