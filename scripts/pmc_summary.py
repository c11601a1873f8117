"""Per-kernel mean of the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
(scripts/pmc.sh) -> JSON.  Units: rocprofv3 reports both in KiB.  gfx950
correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts exactly half the
bytes of wide coalesced reads -> hbm_read_bytes = 2 x FETCH_SIZE; WRITE_SIZE
is exact for 16-B stores.  Both count Infinity-Cache hits too (memory-side
requests of L2), so they bound HBM traffic from above."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.replace("gcnk::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def load(d):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return vals


def main(root):
    out = {}
    for sub in ("fetch", "write"):
        for (k, c), v in load(os.path.join(root, sub)).items():
            if not k.startswith(("spmm_", "gemm_")):
                continue
            out.setdefault(k, {})[c] = {"mean_kib": sum(v) / len(v), "dispatches": len(v)}
    for k, d in out.items():
        f = d.get("FETCH_SIZE", {}).get("mean_kib")
        w = d.get("WRITE_SIZE", {}).get("mean_kib")
        if f is not None and w is not None:
            d["hbm_bytes_per_launch"] = 2 * f * 1024 + w * 1024
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
