#!/usr/bin/env python3
"""Reduce tools/pmc_traffic.sh output to HBM bytes per launch of each bench
leg -> profiles/<name>.json (read by bench.py for roofline.traffic).

Decode legs: every zcg:: dispatch of the leg summed, divided by the number
of decode calls in the pass (warmup 1 + steps 2 = 3).
Encode legs: every dispatch of the encode pipeline (zcg:: kernels and the
hipCUB/rocPRIM radix sorts) summed, divided by the number of encode calls
in the pass (warmup 1 + steps 2 = 3).

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts
wide (16 B/lane) coalesced reads at half their bytes, so it is doubled (an
upper bound for scattered narrow reads); WRITE_SIZE is exact.  The counters
are in KiB."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import ENCODE_LEG, KERNEL, LEG  # noqa: E402

ENCODE_CALLS = 3
DECODE_CALLS = 3  # tools/pmc_traffic.sh runs the decode legs with --warmup 1 --steps 2


def dispatches(path):
    """{dispatch id: (kernel name, counter value)} of one pass."""
    vals = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            name, v = r["Kernel_Name"], float(r["Counter_Value"])
            old = vals.get(key, (name, 0.0))
            vals[key] = (name, old[1] + v)
    return vals


def is_encode_kernel(name):
    return ("zcg::" in name and "raw_kernel" not in name) or "rocprim" in name or "hipcub" in name


def main(src, dst):
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over the bench leg "
                     "(tools/pmc_traffic.sh); bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 "
                     "FETCH_SIZE counts 16 B/lane reads at half)",
           "legs": {}}
    for leg in sorted(os.listdir(src)):
        if not leg.endswith(".FETCH_SIZE"):
            continue
        leg = leg[:-len(".FETCH_SIZE")]
        f = dispatches(os.path.join(src, f"{leg}.FETCH_SIZE"))
        w = dispatches(os.path.join(src, f"{leg}.WRITE_SIZE"))
        if leg.endswith("_encode"):
            fs = sum(v for n, v in f.values() if is_encode_kernel(n)) / ENCODE_CALLS
            ws = sum(v for n, v in w.values() if is_encode_kernel(n)) / ENCODE_CALLS
            kn = sorted({n.split("(")[0] for n, _ in f.values() if is_encode_kernel(n)})
            res["legs"][leg] = {"batch_per_gpu": ENCODE_LEG[leg[:-len("_encode")]][0], "kernels": kn,
                                "fetch_bytes": int(2 * fs * 1024), "write_bytes": int(ws * 1024),
                                "traffic_bytes": int(2 * fs * 1024 + ws * 1024), "per": "encode call"}
            continue
        # every zcg:: dispatch of the leg's decode calls (warmup 1 + steps 2)
        fv = [v for n, v in f.values() if "zcg::" in n]
        wv = [v for n, v in w.values() if "zcg::" in n]
        if not fv or not wv:
            continue
        fm, wm = sum(fv) / DECODE_CALLS, sum(wv) / DECODE_CALLS
        kn = sorted({n.split("(")[0] for n, _ in f.values() if "zcg::" in n})
        batch = LEG[leg]["batch"]
        res["legs"][leg] = {"kernel": KERNEL[leg], "kernels": kn, "batch_per_gpu": batch,
                            "fetch_bytes": int(2 * fm * 1024), "write_bytes": int(wm * 1024),
                            "traffic_bytes": int(2 * fm * 1024 + wm * 1024), "dispatches": len(fv),
                            "per": "decode call"}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
