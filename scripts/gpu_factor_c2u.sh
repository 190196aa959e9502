cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/fac
for f in auto force4 force2; do
  timeout -k 10 300 python bench.py --config config2 --dtype u8 --factor $f --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/fac/c2u_$f.json 2> gpurun_out/fac/c2u_$f.err || { echo "fail $f"; tail -3 gpurun_out/fac/c2u_$f.err; exit 1; }
  python -c "
import json,sys
d=json.loads(open('gpurun_out/fac/c2u_$f.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$f', round(d['ms_per_step'],2), r.get('kernel'), round(r.get('kernel_ms_per_launch',0),2), d['config'].get('method'), d['config']['plan'].get('dms_per_block'))"
done
