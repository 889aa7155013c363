#!/bin/bash
# SQ counters of the LZ4 block kernel on a C4-shaped batch (GPU box).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/lzpmc"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/lzpmc/p$i" -o pmc -- \
    python3 "$R/bench.py" --codec lz4 --global-batch 8192 --pool 256 --steps 1 --warmup 1 --no-extra --no-cpu-baseline \
    > "$R/gpurun_out/lzpmc/p$i.log" 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, os, collections
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
for f in sorted(glob.glob(f"{R}/gpurun_out/lzpmc/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "lz4_blocks_kernel" not in r["Kernel_Name"]: continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f, dict(agg))
PY
