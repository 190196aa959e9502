#!/bin/bash
# Same-build evidence pass on one MI355X: smoke, the GPU suite, bench lines
# and rocprofv3 kernel stats + separate FETCH_SIZE / WRITE_SIZE passes.
#   O=gpurun_out/<dir> PARTS="smoke tests bench prof" BENCH="name|args;..." PROF="name|args;..."
# The source digest of the library (pypulsar_amd._lib.source_digest) is
# written to $O/src_digest.txt; scripts/collect_profiles.py stamps it into
# profiles/pmc_sweep.json so bench.py only uses counters of the same build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=${O:-gpurun_out/ev}
mkdir -p $O
PARTS=${PARTS:-"smoke bench prof"}
timeout -k 10 300 python -c "from pypulsar_amd import _lib; print(_lib.loaded_digest())" > $O/src_digest.txt || exit 1
echo "digest $(cat $O/src_digest.txt)"
run() { local t=$1 n=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -5 $O/$n.err; exit 1; }; echo "$n: $(cut -c1-240 $O/$n.json)"; }
for p in $PARTS; do case $p in
smoke)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.log; exit 1; }
  echo SMOKE_OK ;;
tests)
  timeout -k 10 900 python -u -m pytest ${TFILES:-tests} -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log ;;
bench)
  IFS=';' read -ra L <<< "${BENCH:-config3|;northstar|--config northstar --no-cpu-baseline --no-e2e}"
  for item in "${L[@]}"; do
    name=${item%%|*}; args=${item#*|}
    run ${BT:-600} bench_$name python bench.py $args
  done ;;
prof)
  P=$O/prof
  mkdir -p $P
  IFS=';' read -ra L <<< "${PROF:-config3|--config config3;northstar|--config northstar}"
  for item in "${L[@]}"; do
    name=${item%%|*}; args=${item#*|}
    A="$args --steps 2 --warmup 1 --no-cpu-baseline --no-e2e"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/kt_$name -o kt --output-format csv -- python bench.py $A > $P/kt_$name.log 2>&1 || { echo "kt $name failed"; tail -5 $P/kt_$name.log; exit 1; }
    timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $P/fe_$name -o p --output-format csv -- python bench.py $A > $P/fe_$name.log 2>&1 || { echo "fetch $name failed"; tail -5 $P/fe_$name.log; exit 1; }
    timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $P/wr_$name -o p --output-format csv -- python bench.py $A > $P/wr_$name.log 2>&1 || { echo "write $name failed"; tail -5 $P/wr_$name.log; exit 1; }
    echo "prof $name ok"
  done ;;
esac; done
