#!/bin/bash
# SQ counters of a gzip decode kernel on the C2 bench batch (GPU box).
# usage: tools/inf_pmc.sh [kernel-name substring] (default inflate_wave_kernel)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
K="${1:-inflate_wave_kernel}"
mkdir -p "$R/gpurun_out/infpmc"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/infpmc/p$i" -o pmc -- \
    python3 "$R/bench.py" --codec ${CODEC:-gzip} --steps 1 --warmup 1 --no-extra --no-cpu-baseline \
    > "$R/gpurun_out/infpmc/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/infpmc/p$i.log"; exit 1; }
done
K="$K" python3 - <<'PY'
import csv, glob, os, collections, json
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo"); K = os.environ["K"]
agg = collections.defaultdict(float); calls = collections.Counter()
for f in sorted(glob.glob(f"{R}/gpurun_out/infpmc/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if K not in r["Kernel_Name"]: continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        calls[r["Counter_Name"]] += 1
per = {k: v / max(1, calls[k]) for k, v in sorted(agg.items())}  # per launch
d = {}
if per.get("SQ_WAVE_CYCLES"):
    wc = per["SQ_WAVE_CYCLES"]
    d["wait_any_frac"] = round(per.get("SQ_WAIT_ANY", 0) / wc, 3)
    d["active_inst_any_frac"] = round(per.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3)
    d["valu_insts_per_wave"] = round(per.get("SQ_INSTS_VALU", 0) / max(1, per.get("SQ_WAVES", 1)))
out = {"kernel": K, "per_launch": per, "derived": d}
json.dump(out, open(f"{R}/gpurun_out/infpmc/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
