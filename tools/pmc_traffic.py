#!/usr/bin/env python3
"""Reduce tools/pmc_traffic.sh output to HBM bytes per launch of each bench
leg -> profiles/<name>.json (read by bench.py for roofline.traffic).

Decode legs: every zcg:: dispatch of the leg summed, divided by the number
of decode calls in the pass (warmup 1 + steps 2 = 3).
Encode legs: every dispatch of the encode pipeline (zcg:: kernels and the
hipCUB/rocPRIM radix sorts) summed, divided by the number of encode calls
in the pass (warmup 1 + steps 2 = 3).

gfx950 corrections: the multipliers come from profiles/r05_pmc_calibration.json
(tools/probe/pmc_calib.hip, known byte counts): every L2 read miss leaves as
one 128 B request whatever the access width, and FETCH_SIZE tallies 64 B per
request, so read bytes = 2.0 x FETCH_SIZE for streams and 1/4/16-byte
gathers alike; WRITE_SIZE already counts 64 B / 32 B write requests as issued
(multiplier 1.0).  When the leg's sized-request pass is present the read
bytes are taken from it directly (128*RDREQ_128B + 64*RDREQ_64B +
32*RDREQ_32B) and the FETCH_SIZE figure is kept beside it as the check.
The counters do not separate Infinity-Cache hits (RDREQ_DRAM == RDREQ), so
the figure is fabric traffic, an upper bound on HBM bytes.  FETCH_SIZE /
WRITE_SIZE are in KiB."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import ENCODE_LEG, KERNEL, LEG  # noqa: E402

ENCODE_CALLS = 3
DECODE_CALLS = 3  # tools/pmc_traffic.sh runs the decode legs with --warmup 1 --steps 2


CALIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                     "r05_pmc_calibration.json")


def multipliers():
    """(FETCH_SIZE, WRITE_SIZE) multipliers measured by tools/pmc_calib.py: the
    largest over the calibrated patterns (they agree to 0.05 %)."""
    r = json.load(open(CALIB))["result"]
    return r["fetch_multiplier_range"][1], r["write_multiplier_range"][1]


def dispatches(path, counter=None):
    """{dispatch id: (kernel name, counter value)} of one pass (one counter of
    it when `counter` is given)."""
    vals = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if counter is not None and r["Counter_Name"] != counter:
                continue
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            name, v = r["Kernel_Name"], float(r["Counter_Value"])
            old = vals.get(key, (name, 0.0))
            vals[key] = (name, old[1] + v)
    return vals


def sized_reads(src, leg, keep, calls):
    """Read bytes per call from the leg's TCC_EA0_RDREQ_{32,64,128}B pass, and
    the 128 B share of its requests; None when the pass is absent."""
    d = os.path.join(src, f"{leg}.RDREQ")
    if not os.path.isdir(d):
        return None
    tot, n = 0.0, {}
    for b in (32, 64, 128):
        v = sum(x for k, x in dispatches(d, f"TCC_EA0_RDREQ_{b}B").values() if keep(k))
        n[b] = v
        tot += b * v
    allreq = sum(n.values())
    return tot / calls, (n[128] / allreq if allreq else None)


def is_encode_kernel(name):
    return ("zcg::" in name and "raw_kernel" not in name) or "rocprim" in name or "hipcub" in name


def traffic_row(fetch_kib, write_kib, sized, fm_mul, wm_mul):
    """Traffic fields of one leg from per-call FETCH_SIZE / WRITE_SIZE (KiB)."""
    fb = fm_mul * fetch_kib * 1024
    row = {"fetch_size_bytes": int(fetch_kib * 1024), "fetch_bytes_calibrated": int(fb)}
    if sized is not None:
        row["fetch_bytes_sized_requests"] = int(sized[0])
        row["read_req_128B_share"] = None if sized[1] is None else round(sized[1], 5)
        fb = sized[0]
    wb = wm_mul * write_kib * 1024
    row.update({"fetch_bytes": int(fb), "write_bytes": int(wb), "traffic_bytes": int(fb + wb)})
    return row


def main(src, dst):
    fm_mul, wm_mul = multipliers()
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_EA0_RDREQ_{32,64,128}B in separate passes over "
                     "the bench leg (tools/pmc_traffic.sh); read bytes = sized read requests (128*RDREQ_128B + "
                     "64*RDREQ_64B + 32*RDREQ_32B) when measured, else fetch_multiplier*FETCH_SIZE; write bytes = "
                     "write_multiplier*WRITE_SIZE; multipliers from profiles/r05_pmc_calibration.json",
           "fetch_multiplier": fm_mul, "write_multiplier": wm_mul,
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
            row = {"batch_per_gpu": ENCODE_LEG[leg[:-len("_encode")]][0], "kernels": kn, "per": "encode call"}
            row.update(traffic_row(fs, ws, sized_reads(src, leg, is_encode_kernel, ENCODE_CALLS), fm_mul, wm_mul))
            res["legs"][leg] = row
            continue
        # every zcg:: dispatch of the leg's decode calls (warmup 1 + steps 2)
        fv = [v for n, v in f.values() if "zcg::" in n]
        wv = [v for n, v in w.values() if "zcg::" in n]
        if not fv or not wv:
            continue
        fm, wm = sum(fv) / DECODE_CALLS, sum(wv) / DECODE_CALLS
        kn = sorted({n.split("(")[0] for n, _ in f.values() if "zcg::" in n})
        batch = LEG[leg]["batch"]
        row = {"kernel": KERNEL[leg], "kernels": kn, "batch_per_gpu": batch, "dispatches": len(fv),
               "per": "decode call"}
        row.update(traffic_row(fm, wm, sized_reads(src, leg, lambda n: "zcg::" in n, DECODE_CALLS), fm_mul, wm_mul))
        res["legs"][leg] = row
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
