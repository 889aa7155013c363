#!/usr/bin/env python3
"""Reduce tools/pmc_calib.sh output -> profiles/<name>.json: per access
pattern, what each counter reports against the KNOWN bytes of the pattern.

For every pattern the probe touches each unit of a 1 GiB buffer exactly once
in a scattered order after an eviction pass, so:
  - reads: the distinct 128 B lines touched (`lines128`) is the least the
    memory side can move; `fetch_per_line` = FETCH_SIZE bytes / lines,
    `fetch_factor` = accessed bytes / FETCH_SIZE bytes (what FETCH_SIZE must be
    multiplied by to give the bytes the kernel asked for);
  - writes: `write_factor` = written bytes / WRITE_SIZE bytes.
The request counters (TCC_EA0_RDREQ, _32B, _DRAM; TCC_EA0_WRREQ, _64B) are
reported per line / per access as measured, so the units are visible.
  usage: pmc_calib.py SRC_DIR OUT_JSON"""
import csv
import glob
import json
import os
import sys


def per_kernel(path, vals):
    """Adds {counter: {kernel name prefix 'calib_k<M': value}} of one pass to vals."""
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "calib_k<" not in name:
                continue
            m = name[name.index("calib_k<"):].split(",")[0]
            c = vals.setdefault(r["Counter_Name"], {})
            c[m] = c.get(m, 0.0) + float(r["Counter_Value"])


def main(src, dst):
    pats = [json.loads(l) for l in open(os.path.join(src, "plain.jsonl")) if l.startswith("{")]
    meas = {}
    for d in sorted(os.listdir(src)):
        if os.path.isdir(os.path.join(src, d)):
            per_kernel(os.path.join(src, d), meas)
    counters = sorted(meas)
    t33 = {}
    if os.path.exists(os.path.join(src, "plain33.jsonl")):
        t33 = {q["pattern"]: q for q in map(json.loads, open(os.path.join(src, "plain33.jsonl"))) if q}
    out = {"method": "tools/probe/pmc_calib.hip under tools/pmc_calib.sh: one rocprofv3 --pmc pass per counter; "
                     "each pattern touches every unit of a 1 GiB buffer once in a scattered order after a 512 MiB "
                     "eviction write; FETCH_SIZE / WRITE_SIZE are in KiB, TCC_EA0_* are request counts",
           "patterns": {}}
    for p in pats:
        k = p["kernel"]
        row = {x: p[x] for x in ("kind", "what", "buffer_bytes", "units", "unit_bytes", "width", "accessed_bytes",
                                 "lines128", "ms")}
        row["counters"] = {c: meas[c].get(k) for c in counters}
        if p["pattern"] in t33:
            row["ms_8GiB"] = t33[p["pattern"]]["ms"]
        r32, r64, r128 = (meas.get(f"TCC_EA0_RDREQ_{b}B", {}).get(k) for b in (32, 64, 128))
        if None not in (r32, r64, r128):
            rb = 32 * r32 + 64 * r64 + 128 * r128
            row["rdreq_sized_bytes"] = int(rb)
            if p["kind"] == "read":
                row["rdreq_sized_per_line128"] = round(rb / p["lines128"], 3)
        f, w = meas.get("FETCH_SIZE", {}).get(k), meas.get("WRITE_SIZE", {}).get(k)
        if p["kind"] == "read" and f:
            fb = f * 1024
            row["fetch_bytes"] = int(fb)
            row["fetch_per_line128"] = round(fb / p["lines128"], 3)
            row["fetch_factor"] = round(p["accessed_bytes"] / fb, 4)
            if "rdreq_sized_bytes" in row:
                # what FETCH_SIZE must be multiplied by to give the bytes the
                # memory side moved (sized read requests)
                row["fetch_multiplier"] = round(row["rdreq_sized_bytes"] / fb, 4)
            for c in ("TCC_EA0_RDREQ", "TCC_EA0_RDREQ_32B", "TCC_EA0_RDREQ_DRAM"):
                v = meas.get(c, {}).get(k)
                if v is not None:
                    row[c + "_per_line128"] = round(v / p["lines128"], 3)
        if p["kind"] == "write" and w:
            wb = w * 1024
            row["write_bytes"] = int(wb)
            row["write_factor"] = round(p["accessed_bytes"] / wb, 4)
            q, q64 = meas.get("TCC_EA0_WRREQ", {}).get(k), meas.get("TCC_EA0_WRREQ_64B", {}).get(k)
            if q is not None and q64 is not None:
                row["wrreq_sized_bytes"] = int(64 * q64 + 32 * (q - q64))
                row["write_multiplier"] = round(row["wrreq_sized_bytes"] / wb, 4)
            for c in ("TCC_EA0_WRREQ", "TCC_EA0_WRREQ_64B"):
                v = meas.get(c, {}).get(k)
                if v is not None:
                    row[c + "_per_64B"] = round(v / (p["accessed_bytes"] / 64), 3)
        out["patterns"][p["pattern"]] = row
    rm = [r["fetch_multiplier"] for r in out["patterns"].values() if "fetch_multiplier" in r]
    wm = [r["write_multiplier"] for r in out["patterns"].values() if "write_multiplier" in r]
    out["result"] = {
        "fetch_multiplier_range": [min(rm), max(rm)] if rm else None,
        "write_multiplier_range": [min(wm), max(wm)] if wm else None,
        "reads": "every L2 read miss leaves as ONE 128 B request (TCC_EA0_RDREQ_128B == TCC_EA0_RDREQ, _32B = _64B = 0) "
                 "whatever the access width (1/4/16 B, aligned or straddling a line); FETCH_SIZE tallies 64 B per "
                 "request, so memory-side read bytes = 2 x FETCH_SIZE for every pattern measured, gathers included. "
                 "A narrow gather that misses moves a whole 128 B line: 128/width x its useful bytes",
        "writes": "WRITE_SIZE = 64 B per 64 B request + 32 B per smaller request (TCC_EA0_WRREQ_64B vs TCC_EA0_WRREQ): "
                  "it is the memory-side write bytes as issued; a scattered 16 B store costs 32 B, a 4 B store 32 B, "
                  "a 64 B piece (4 lanes x 16 B) or a coalesced stream is exact",
        "infinity_cache": "TCC_EA0_RDREQ_DRAM == TCC_EA0_RDREQ on every pattern: the counters do not separate "
                          "Infinity-Cache hits, so traffic is fabric (L2 -> memory side) bytes, an upper bound on HBM",
        "applied": "tools/pmc_traffic.py: traffic = fetch_multiplier x FETCH_SIZE + write_multiplier x WRITE_SIZE per "
                   "leg, multipliers from this file; each leg's own TCC_EA0_RDREQ_{32,64,128}B pass checks the "
                   "128 B request assumption on the leg itself",
    }
    json.dump(out, open(dst, "w"), indent=1)
    for n, r in out["patterns"].items():
        print(f"{n:20s} {r['ms']:9.3f} ms  " +
              "  ".join(f"{c}={v:.4g}" for c, v in r.items()
                        if c.endswith(("factor", "multiplier", "per_line128", "per_64B"))))
    print(out["result"]["fetch_multiplier_range"], out["result"]["write_multiplier_range"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
