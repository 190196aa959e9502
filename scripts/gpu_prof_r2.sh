#!/bin/bash
# rocprofv3 evidence for the bench lines: kernel trace + stats, then separate
# PMC passes FETCH_SIZE and WRITE_SIZE (never combined with tracing), for each
# configuration in CFGS ("name:extra bench args").
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/prof_r2
mkdir -p $O
CFGS=${CFGS:-"config3:--config config3" "config2_u8:--config config2 --dtype u8" "config2_f32:--config config2 --dtype f32"}
for cfg in "${CFGS[@]}"; do :; done
IFS=';' read -ra L <<< "${CFGL:-config3|--config config3;config2_u8|--config config2 --dtype u8;config2_f32|--config config2 --dtype f32}"
for item in "${L[@]}"; do
  name=${item%%|*}; args=${item#*|}
  A="$args --steps 2 --warmup 1 --no-cpu-baseline"
  echo "== $name $(date +%T)"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_$name -o kt --output-format csv -- python bench.py $A > $O/kt_$name.log 2>&1 || { echo "kt $name failed"; tail -5 $O/kt_$name.log; exit 1; }
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/fe_$name -o p --output-format csv -- python bench.py $A > $O/fe_$name.log 2>&1 || { echo "fetch $name failed"; tail -5 $O/fe_$name.log; exit 1; }
  timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $O/wr_$name -o p --output-format csv -- python bench.py $A > $O/wr_$name.log 2>&1 || { echo "write $name failed"; tail -5 $O/wr_$name.log; exit 1; }
done
echo PROFILE_OK
