#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (sqlite .db or
kernel_stats.csv) into a small committed text file under profiles/."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = list(c.execute("select name,total_calls,total_duration,average,percentage from top_kernels"))
    meta = {}
    for r in c.execute("select name, vgpr_count, sgpr_count, lds_size, scratch_size, grid_x, workgroup_x "
                       "from kernels group by name"):
        meta[r[0]] = r[1:]
    return rows, meta


def main(src, out, note=""):
    dbs = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
    rows, meta = from_db(dbs[0])
    with open(out, "w") as f:
        f.write(f"# rocprofv3 --kernel-trace --stats summary ({note})\n")
        f.write("# durations in milliseconds (rocpd top_kernels view reports microseconds; /1000)\n")
        f.write("name | calls | total_ms | avg_ms | pct | vgpr | sgpr | lds | scratch | grid_x | wg_x\n")
        for r in rows:
            m = meta.get(r[0], ("", "", "", "", "", ""))
            name = r[0][:110]
            f.write(f"{name} | {r[1]} | {r[2]/1000:.1f} | {r[3]/1000:.1f} | {r[4]:.2f} | "
                    + " | ".join(str(x) for x in m) + "\n")
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], " ".join(sys.argv[3:]))
