#!/bin/bash
# Fabric traffic of the inflate wave kernel split by access class (GPU box):
# WRITE_SIZE and the sized read requests (TCC_EA0_RDREQ_{32,64,128}B) of the
# C2 batch (tools/iw_traffic.py) for the product build and the ablation
# builds of tools/iw_ablate.py, one rocprofv3 --pmc pass per counter group,
# each under its own time limit; the first failure ends the script.
#   usage: tools/iw_traffic_split.sh OUTDIR [variant ...]   (in-tree = product)
set -o pipefail
out=$(realpath -m "$1"); shift
root="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for v in in-tree "$@"; do
  if [ "$v" = in-tree ]; then unset ZCG_LIB; else export ZCG_LIB=$root/variants/$v.so; fi
  for k in WRITE_SIZE "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B"; do
    d=${k%% *}; [ "$d" = TCC_EA0_RDREQ ] && d=RDREQ
    timeout -s KILL 240 rocprofv3 --pmc $k --output-format csv -d "$out/$v.$d" -o pmc -- \
      python3 "$root/tools/iw_traffic.py" > "$out/$v.$d.log" 2>&1 || { echo "$v $d failed"; tail -5 "$out/$v.$d.log"; exit 1; }
    tail -1 "$out/$v.$d.log"
  done
done
python3 - "$out" in-tree "$@" <<'PY'
import csv, glob, json, os, sys
out, names = sys.argv[1], sys.argv[2:]
res = {}
for v in names:
    r = {}
    for d in ("WRITE_SIZE", "RDREQ"):
        acc, disp = {}, set()
        for f in glob.glob(f"{out}/{v}.{d}/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                if "inflate_wave_kernel" not in row["Kernel_Name"]:
                    continue
                disp.add(row["Dispatch_Id"])
                acc[row["Counter_Name"]] = acc.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
        nd = max(1, len(disp))
        for k, x in acc.items():
            r[k] = x / nd
        r[d + "_dispatches"] = len(disp)
    rd = 128 * r.get("TCC_EA0_RDREQ_128B", 0) + 64 * r.get("TCC_EA0_RDREQ_64B", 0) + 32 * r.get("TCC_EA0_RDREQ_32B", 0)
    res[v] = {"read_bytes": rd, "write_bytes": 1024 * r.get("WRITE_SIZE", 0), "raw": r,
              "run": open(f"{out}/{v}.RDREQ.log").read().strip().splitlines()[-1]}
json.dump(res, open(f"{out}/split.json", "w"), indent=1)
print(json.dumps({k: {"read_GB": round(v["read_bytes"] / 1e9, 2), "write_GB": round(v["write_bytes"] / 1e9, 2)} for k, v in res.items()}))
PY
