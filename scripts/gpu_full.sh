#!/bin/bash
# Full GPU round: smoke, GPU parity suite, bench (f32 + u8), rocprofv3 kernel
# trace/stats and separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/full
mkdir -p $O
BA="--steps 5 --warmup 2 --no-cpu-baseline"
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo PYTEST_OK \
 && timeout -k 10 600 python bench.py > $O/bench_f32.json 2> $O/bench_f32.err && echo BENCH_F32_OK \
 && timeout -k 10 300 python bench.py --dtype u8 --no-cpu-baseline > $O/bench_u8.json 2> $O/bench_u8.err && echo BENCH_U8_OK \
 && timeout -k 10 300 python bench.py --config stream --steps 6 --warmup 2 > $O/bench_stream.json 2> $O/bench_stream.err && echo BENCH_STREAM_OK \
 && timeout -k 10 300 python bench.py --config subband --steps 3 --warmup 1 > $O/bench_subband.json 2> $O/bench_subband.err && echo BENCH_SUBBAND_OK \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_stream -o kt --output-format csv -- python bench.py --config stream --steps 4 --warmup 1 > $O/kt_stream.log 2>&1 \
 && timeout -k 10 300 python bench.py --config search --steps 5 --warmup 2 > $O/bench_search.json 2> $O/bench_search.err && echo BENCH_SEARCH_OK \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_search -o kt --output-format csv -- python bench.py --config search --steps 5 --warmup 2 > $O/kt_search.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_subband -o kt --output-format csv -- python bench.py --config subband --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_subband.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_f32 -o kt --output-format csv -- python bench.py $BA > $O/kt_f32.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_u8 -o kt --output-format csv -- python bench.py $BA --dtype u8 > $O/kt_u8.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_f32 -o p --output-format csv -- python bench.py $BA > $O/pmc1.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_f32 -o p --output-format csv -- python bench.py $BA > $O/pmc2.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_u8 -o p --output-format csv -- python bench.py $BA --dtype u8 > $O/pmc3.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_u8 -o p --output-format csv -- python bench.py $BA --dtype u8 > $O/pmc4.log 2>&1 \
 && echo PROFILE_OK
rc=$?
tail -3 $O/pytest_gpu.log
cat $O/bench_f32.json $O/bench_u8.json $O/bench_stream.json $O/bench_subband.json 2>/dev/null | cut -c1-300
exit $rc
