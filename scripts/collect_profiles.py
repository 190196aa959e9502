"""Copy the judged evidence of a scripts/gpu_full.sh run from gpurun_out/full
into profiles/: the rocprofv3 kernel-stats summaries, the bench lines, and the
per-launch HBM-side traffic of the sweep kernel from the separate FETCH_SIZE /
WRITE_SIZE passes (profiles/pmc_sweep.json, read by bench.py).

FETCH_SIZE is doubled: on gfx950 it reports half of the bytes of 16-B/lane
streaming reads, which is what the sweep's global_load_lds_dwordx4 staging is
(MI355X_MICROARCH.md, HBM/rocprofv3 section); WRITE_SIZE is exact for
16-B-per-lane and dword streaming stores.  Both count L2 <-> fabric traffic
(Infinity Cache hits included)."""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "full")
DST = os.path.join(ROOT, "profiles")
TAG = sys.argv[1] if len(sys.argv) > 1 else "r1"


def per_kernel(pattern, counter):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                out[r["Kernel_Name"].split("(")[0]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in out.items()}


def main():
    os.makedirs(DST, exist_ok=True)
    for name in ("f32", "u8", "stream", "subband", "search"):
        f = glob.glob(os.path.join(SRC, "kt_" + name, "**", "*kernel_stats.csv"), recursive=True)
        if f:
            shutil.copy(f[0], os.path.join(DST, "%s_%s_kernel_stats.csv" % (TAG, name)))
    for name in ("f32", "u8", "stream", "subband", "search"):
        f = os.path.join(SRC, "bench_%s.json" % name)
        if os.path.exists(f):
            lines = [l for l in open(f) if l.startswith("{")]
            if lines:
                open(os.path.join(DST, "%s_bench_%s.json" % (TAG, name)), "w").write(lines[-1])
    pmc = {}
    for dt in ("f32", "u8"):
        fe = per_kernel(os.path.join(SRC, "pmc_fetch_" + dt, "**", "*counter_collection.csv"),
                        "FETCH_SIZE")
        wr = per_kernel(os.path.join(SRC, "pmc_write_" + dt, "**", "*counter_collection.csv"),
                        "WRITE_SIZE")
        k = [n for n in fe if "k_sweep" in n]
        if not k:
            continue
        k = k[0]
        fkb, launches = fe[k]
        wkb = wr.get(k, (0.0, 0))[0]
        pmc["config2_" + dt] = {
            "kernel": k,
            "fetch_size_kb_per_launch": fkb,
            "write_size_kb_per_launch": wkb,
            "launches": launches,
            "hbm_bytes_per_launch": 2 * fkb * 1024 + wkb * 1024,
            "note": "separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `python bench.py "
                    "--steps 5 --warmup 2 --no-cpu-baseline%s`; bytes = 2 x FETCH_SIZE (gfx950 "
                    "reports half of 16-B/lane streaming reads) + WRITE_SIZE, KB x 1024"
                    % ("" if dt == "f32" else " --dtype u8"),
        }
    if pmc:
        json.dump(pmc, open(os.path.join(DST, "pmc_sweep.json"), "w"), indent=1)
    print("profiles:", sorted(os.listdir(DST)))
    print(json.dumps(pmc, indent=1))


if __name__ == "__main__":
    main()
