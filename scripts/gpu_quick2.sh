#!/bin/bash
# GPU parity suite + config-2 bench (f32, u8) + kernel stats of the f32 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/q2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo PYTEST_OK \
 && timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_f32.json 2> $O/bench_f32.err && echo F32_OK \
 && timeout -k 10 300 python bench.py --dtype u8 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_u8.json 2> $O/bench_u8.err && echo U8_OK \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_f32 -o kt --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/kt_f32.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_u8 -o kt --output-format csv -- python bench.py --dtype u8 --steps 5 --warmup 2 --no-cpu-baseline > $O/kt_u8.log 2>&1 && echo PROF_OK
rc=$?
tail -3 $O/pytest_gpu.log
for f in $O/bench_f32.json $O/bench_u8.json; do python -c "import json;d=json.load(open('$f'));print(d['dtype'],round(d['ms_per_step'],2),round(d['roofline']['kernel_ms'],2))"; done
grep -h interleave $O/kt_*/kt_kernel_stats.csv | cut -d, -f1-4 | cut -c1-30,150-
exit $rc
