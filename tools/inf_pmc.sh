#!/bin/bash
# SQ counters of the inflate kernel on the C2 bench batch (GPU box).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/infpmc"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/infpmc/p$i" -o pmc -- \
    python3 "$R/bench.py" --codec gzip --steps 1 --warmup 1 --no-extra --no-cpu-baseline \
    > "$R/gpurun_out/infpmc/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/infpmc/p$i.log"; }
done
python3 - <<'PY'
import csv, glob, os, collections
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
agg = collections.defaultdict(float); calls = collections.Counter()
for f in sorted(glob.glob(f"{R}/gpurun_out/infpmc/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "inflate_par_kernel" not in r["Kernel_Name"]: continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        calls[r["Counter_Name"]] += 1
print({k: (v, calls[k]) for k, v in sorted(agg.items())})
PY
