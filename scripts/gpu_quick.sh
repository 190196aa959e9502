#!/bin/bash
# Quick A/B on the working tree's libpdd: selected GPU tests, then bench lines
# (kernel ms per launch).  TESTK: pytest -k expression; BENCHES: "name|args;...".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/quick
mkdir -p $O
if [ -n "$TESTK" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTK" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
IFS=';' read -ra L <<< "${BENCHES:-config3|--config config3;config2_f32|--config config2;config2_u8|--config config2 --dtype u8}"
for item in "${L[@]}"; do
  name=${item%%|*}; args=${item#*|}
  timeout -k 10 300 python bench.py $args --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-e2e > $O/b_$name.json 2> $O/b_$name.err || { echo "bench $name failed"; tail -3 $O/b_$name.err; exit 1; }
  echo "$name $(python -c "import json;d=json.load(open('$O/b_$name.json'));r=d['roofline'];print('%.2f ms/step' % d['ms_per_step'], r['kernel_ms_per_launch'], r['launches_per_step'], '%.3f' % r['frac'])")"
done
