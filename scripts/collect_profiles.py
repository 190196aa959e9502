"""Copy the judged evidence of scripts/gpu_evidence.sh (prof part) from
gpurun_out/<RUN>/prof into profiles/: rocprofv3 kernel-stats summaries and
the per-launch HBM-side traffic of the sweep kernels
(profiles/pmc_sweep.json, read by bench.py).

Every pmc_sweep.json entry is stamped with the source digest of the library
the run measured (gpurun_out/<RUN>/src_digest.txt, written on the GPU box by
gpu_evidence.sh), the git commit whose sources have that digest (HEAD, when
the working tree's digest matches; else null), the kernel name and the sweep
plan the bench line reported.  bench.py only reports `traffic` when the
digest and plan match the build it runs.

FETCH_SIZE is doubled: on gfx950 it reports half of the bytes of 16-B/lane
streaming reads, which is what the sweep's global_load_lds_dwordx4 staging is
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B-per-lane and
dword streaming stores.  Both count L2 <-> fabric traffic (Infinity Cache hits
included).

Usage: python scripts/collect_profiles.py RUN TAG   (e.g. r4a r4a)
"""
import collections
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
RUN = sys.argv[1]
TAG = sys.argv[2] if len(sys.argv) > 2 else RUN
SRC = os.path.join(ROOT, "gpurun_out", RUN, "prof")
DST = os.path.join(ROOT, "profiles")
# profile name -> pmc_sweep.json key of its sweep kernel (bench.py pmc_key)
KEYS = {"config3": "config3_u8", "config3_channel": "config3_channel", "northstar": "northstar",
        "config2_u8": "config2_u8", "config2_f32": "config2_f32", "stream": "stream"}


def per_kernel(pattern, counter):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                out[r["Kernel_Name"].split("(")[0]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in out.items()}


def bench_line(log):
    try:
        for ln in open(log):
            if ln.startswith("{") and '"metric"' in ln:
                return json.loads(ln)
    except OSError:
        pass
    return None


def main():
    from pypulsar_amd._digest import source_digest
    digest = open(os.path.join(ROOT, "gpurun_out", RUN, "src_digest.txt")).read().strip()
    commit = None
    if source_digest() == digest:
        commit = subprocess.check_output(["git", "rev-parse", "--short", "HEAD"], cwd=ROOT).decode().strip()
    path = os.path.join(DST, "pmc_sweep.json")
    pmc = json.load(open(path)) if os.path.exists(path) else {}
    for kt in sorted(glob.glob(os.path.join(SRC, "kt_*"))):
        if not os.path.isdir(kt):
            continue
        name = os.path.basename(kt)[3:]
        f = glob.glob(os.path.join(kt, "**", "*kernel_stats.csv"), recursive=True)
        if f:
            shutil.copy(f[0], os.path.join(DST, "%s_%s_kernel_stats.csv" % (TAG, name)))
        line = bench_line(os.path.join(SRC, "kt_%s.log" % name)) or {}
        plan = line.get("config", {}).get("plan")
        method = line.get("config", {}).get("method")
        # the run the counters belong to: bench.py reports traffic only for a
        # line of the same mode, world size and launches per step (columns
        # per launch)
        ctx = {"mode": line.get("config", {}).get("mode"), "world": line.get("n_gpus"),
               "launches_per_step": (line.get("roofline") or {}).get("launches_per_step")}
        fe = per_kernel(os.path.join(SRC, "fe_" + name, "**", "*counter_collection.csv"), "FETCH_SIZE")
        wr = per_kernel(os.path.join(SRC, "wr_" + name, "**", "*counter_collection.csv"), "WRITE_SIZE")
        key = KEYS.get(name, name)
        stamp = {"round": TAG, "src_digest": digest, "commit": commit, "plan": plan, "method": method,
                 "ctx": ctx}
        for n1 in fe:
            if "k_fx_patterns" in n1:
                pmc[key + "_stage1"] = dict(
                    kernel=n1, fetch_size_kb_per_launch=fe[n1][0],
                    write_size_kb_per_launch=wr.get(n1, (0.0, 0))[0], launches=fe[n1][1],
                    hbm_bytes_per_launch=2 * fe[n1][0] * 1024 + wr.get(n1, (0.0, 0))[0] * 1024, **stamp)
        k = [n for n in fe if "k_sweep_il" in n]
        if not k:
            continue
        k = max(k, key=lambda n: fe[n][1])
        fkb, launches = fe[k]
        wkb = wr.get(k, (0.0, 0))[0]
        pmc[key] = dict(
            kernel=k, fetch_size_kb_per_launch=fkb, write_size_kb_per_launch=wkb, launches=launches,
            hbm_bytes_per_launch=2 * fkb * 1024 + wkb * 1024,
            note="separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the profiled bench "
                 "command (scripts/gpu_evidence.sh, --steps 2 --warmup 1); bytes = 2 x FETCH_SIZE "
                 "(gfx950 reports half of 16-B/lane streaming reads) + WRITE_SIZE, KB x 1024", **stamp)
    json.dump(pmc, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: (v.get("kernel"), v.get("hbm_bytes_per_launch"), v.get("round"))
                      for k, v in pmc.items()}, indent=1))


if __name__ == "__main__":
    main()
