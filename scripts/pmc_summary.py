"""Summarise rocprofv3 --pmc CSVs under a directory: per (pass, kernel), the
mean over the kernel's dispatches of every counter (summed over instances)."""
import collections
import csv
import glob
import os
import sys


def main(root):
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r.get("Kernel_Name", "?")
                if "pdd" not in k:
                    continue
                acc[k.split("(")[0][:70]][r["Counter_Name"]][r.get("Dispatch_Id")] += float(r["Counter_Value"])
        print("==", os.path.relpath(f, root))
        for k, ctrs in acc.items():
            print("  ", k)
            for c, per in sorted(ctrs.items()):
                m = sum(per.values()) / max(1, len(per))
                print("     %-24s %.4e  (%d dispatches)" % (c, m, len(per)))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
