cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
for V in 0 2; do
  PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_VARIANT=$V SETS="--config config3" bash scripts/gpu_bench_set.sh || exit 1
  PDD_DEV_LIB=build/libpdd_dev.so PDD_SWEEP_VARIANT=$V timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/exp/fe$V -o p --output-format csv -- python bench.py --config config3 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/exp/fe$V.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv,glob,collections
for V in (0,2):
    agg=collections.defaultdict(list)
    for f in glob.glob('gpurun_out/exp/fe%d/**/*counter_collection.csv'%V, recursive=True):
        for r in csv.DictReader(open(f)):
            if 'sweep' in r['Kernel_Name']: agg[r['Dispatch_Id']].append(float(r['Counter_Value']))
    vals=[sum(v) for v in agg.values()]
    print('variant',V,'FETCH_SIZE KB per launch', sum(vals)/len(vals) if vals else None, len(vals))
PY
