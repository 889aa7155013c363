#!/usr/bin/env python3
"""Reduce tools/pmc_traffic.sh output to HBM bytes per launch of each
codec's bench kernel -> profiles/<name>.json (read by bench.py for
roofline.traffic).

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts
wide (16 B/lane) coalesced reads at half their bytes, so it is doubled;
WRITE_SIZE is exact for 16 B/lane stores.  The counters are in KiB."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import KERNEL  # noqa: E402


BATCH = {"gzip": 4096, "lz4": 4096, "raw": 1024, "xz": 2048, "bzip2": 2048}  # tools/pmc_traffic.sh


def per_dispatch(path, kname):
    vals = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if not r["Kernel_Name"].startswith(kname.split("(")[0].replace("void ", "")) and \
                    kname not in r["Kernel_Name"]:
                continue
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return sorted(vals.values())


def main(src, dst):
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over "
                     "`bench.py --codec C --steps 2 --warmup 1 --no-extra --no-cpu-baseline`; "
                     "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per dispatch (gfx950 FETCH_SIZE "
                     "counts 16 B/lane reads at half), median over the leg's dispatches",
           "kernels": {}}
    for codec, k in KERNEL.items():
        f = per_dispatch(os.path.join(src, f"{codec}.FETCH_SIZE"), k)
        w = per_dispatch(os.path.join(src, f"{codec}.WRITE_SIZE"), k)
        if not f or not w:
            continue
        fm, wm = f[len(f) // 2], w[len(w) // 2]
        res["kernels"][k] = {"codec": codec, "batch_per_gpu": BATCH[codec], "fetch_bytes": int(2 * fm * 1024),
                             "write_bytes": int(wm * 1024), "traffic_bytes": int(2 * fm * 1024 + wm * 1024),
                             "dispatches": len(f)}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
