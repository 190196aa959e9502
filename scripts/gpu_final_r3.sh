#!/bin/bash
# End-of-round-3 evidence: smoke, the GPU suite, every bench line (configs[3]
# default with the CPU baseline and the PCIe leg; the other configs; the
# 8-rank rehearsal), then rocprofv3 kernel stats + separate FETCH_SIZE /
# WRITE_SIZE passes for the sweep lines.  Copy with
# scripts/collect_profiles_r3.py.  PARTS (default "tests bench prof").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/final3}
mkdir -p $O
PARTS=${PARTS:-"tests bench prof"}
run() { local t=$1 n=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -5 $O/$n.err; exit 1; }; echo "$n: $(cut -c1-200 $O/$n.json)"; }
for p in $PARTS; do case $p in
tests)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.log; exit 1; }
  echo SMOKE_OK
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log ;;
bench)
  run 900 bench_config3 python bench.py
  run 600 bench_config3_channel python bench.py --factor off --no-cpu-baseline --no-e2e
  run 300 bench_config2_f32 python bench.py --config config2 --no-cpu-baseline
  run 300 bench_config2_u8 python bench.py --config config2 --dtype u8 --no-cpu-baseline
  run 600 bench_northstar python bench.py --config northstar --no-cpu-baseline --no-e2e
  run 600 bench_northstar_channel python bench.py --config northstar --factor off --no-cpu-baseline --no-e2e
  run 300 bench_stream_wrap python bench.py --config stream --zdm wrap
  run 300 bench_stream_int python bench.py --config stream --zdm int
  run 300 bench_subband python bench.py --config subband
  run 300 bench_search python bench.py --config search
  run 300 bench_ops python bench.py --config ops
  run 600 rehearse8 python bench.py --rehearse 8 ;;
prof)
  P=$O/prof
  mkdir -p $P
  IFS=';' read -ra L <<< "${CFGL:-config3|--config config3;config2_u8|--config config2 --dtype u8;config2_f32|--config config2 --dtype f32;stream|--config stream}"
  for item in "${L[@]}"; do
    name=${item%%|*}; args=${item#*|}
    A="$args --steps 2 --warmup 1 --no-cpu-baseline --no-e2e"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/kt_$name -o kt --output-format csv -- python bench.py $A > $P/kt_$name.log 2>&1 || { echo "kt $name failed"; tail -5 $P/kt_$name.log; exit 1; }
    timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $P/fe_$name -o p --output-format csv -- python bench.py $A > $P/fe_$name.log 2>&1 || { echo "fetch $name failed"; tail -5 $P/fe_$name.log; exit 1; }
    timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $P/wr_$name -o p --output-format csv -- python bench.py $A > $P/wr_$name.log 2>&1 || { echo "write $name failed"; tail -5 $P/wr_$name.log; exit 1; }
    echo "prof $name ok"
  done ;;
esac; done
