"""Copy the judged evidence of scripts/gpu_final_r3.sh (prof part) from
gpurun_out/final3/prof into profiles/: rocprofv3 kernel-stats summaries and the per-launch HBM-side
traffic of the sweep kernel (profiles/pmc_sweep.json, read by bench.py).

FETCH_SIZE is doubled: on gfx950 it reports half of the bytes of 16-B/lane
streaming reads, which is what the sweep's global_load_lds_dwordx4 staging is
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B-per-lane and
dword streaming stores.  Both count L2 <-> fabric traffic (Infinity Cache hits
included)."""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", os.environ.get("FINAL", "final3"), "prof")
DST = os.path.join(ROOT, "profiles")
TAG = sys.argv[1] if len(sys.argv) > 1 else "r3final"
ARGS = {"config3": "--config config3", "config3_channel": "--config config3 --factor off",
        "northstar": "--config northstar", "config2_u8": "--config config2 --dtype u8",
        "config2_f32": "--config config2 --dtype f32", "stream": "--config stream"}


def per_kernel(pattern, counter):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                out[r["Kernel_Name"].split("(")[0]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in out.items()}


def main():
    path = os.path.join(DST, "pmc_sweep.json")
    pmc = json.load(open(path)) if os.path.exists(path) else {}
    for name, args in ARGS.items():
        f = glob.glob(os.path.join(SRC, "kt_" + name, "**", "*kernel_stats.csv"), recursive=True)
        if f:
            shutil.copy(f[0], os.path.join(DST, "%s_%s_kernel_stats.csv" % (TAG, name)))
        fe = per_kernel(os.path.join(SRC, "fe_" + name, "**", "*counter_collection.csv"), "FETCH_SIZE")
        wr = per_kernel(os.path.join(SRC, "wr_" + name, "**", "*counter_collection.csv"), "WRITE_SIZE")
        # factorised plans: the stage-1 pattern kernel's traffic beside the sweep's
        for n1 in fe:
            if "k_fx_patterns" in n1:
                key1 = ("config3_u8" if name == "config3" else name) + "_stage1"
                pmc[key1] = {"kernel": n1, "fetch_size_kb_per_launch": fe[n1][0],
                             "write_size_kb_per_launch": wr.get(n1, (0.0, 0))[0],
                             "launches": fe[n1][1],
                             "hbm_bytes_per_launch": 2 * fe[n1][0] * 1024 + wr.get(n1, (0.0, 0))[0] * 1024,
                             "round": TAG}
        k = [n for n in fe if "k_sweep" in n]
        if not k:
            continue
        k = k[0]
        fkb, launches = fe[k]
        wkb = wr.get(k, (0.0, 0))[0]
        key = name if name != "config3" else "config3_u8"
        pmc[key] = {
            "kernel": k, "fetch_size_kb_per_launch": fkb, "write_size_kb_per_launch": wkb,
            "launches": launches, "hbm_bytes_per_launch": 2 * fkb * 1024 + wkb * 1024,
            "round": TAG,
            "note": "separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `python bench.py "
                    "%s --steps 2 --warmup 1 --no-cpu-baseline --no-e2e`; bytes = 2 x FETCH_SIZE (gfx950 "
                    "reports half of 16-B/lane streaming reads) + WRITE_SIZE, KB x 1024" % args,
        }
    json.dump(pmc, open(path, "w"), indent=1)
    print(json.dumps(pmc, indent=1))


if __name__ == "__main__":
    main()
