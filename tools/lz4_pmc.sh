#!/bin/bash
# SQ counters of an LZ4 block kernel on a C4-shaped batch (GPU box).
#   tools/lz4_pmc.sh [kernel substring] [global batch] [variant ...]
#   (variant: variants/<name>.so via ZCG_LIB; none = the in-tree library)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
K=${1:-lz4_lanes_kernel}; B=${2:-8192}; shift 2 2>/dev/null
VS=${*:-intree}
cd /tmp && export TMPDIR=/tmp
for v in $VS; do
  mkdir -p "$R/gpurun_out/lzpmc/$v"
  if [ "$v" = intree ]; then unset ZCG_LIB; else export ZCG_LIB=$R/variants/$v.so; fi
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY" \
             "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/lzpmc/$v/p$i" -o pmc -- \
      python3 "$R/bench.py" --codec lz4 --global-batch $B --pool 256 --steps 1 --warmup 1 --no-extra --no-cpu-baseline \
      > "$R/gpurun_out/lzpmc/$v/p$i.log" 2>&1 || exit $?
  done
done
python3 - "$K" $VS <<'PY'
import csv, glob, os, collections, sys, json
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
k = sys.argv[1]
for v in sys.argv[2:]:
    agg = collections.defaultdict(float); calls = collections.Counter()
    for f in sorted(glob.glob(f"{R}/gpurun_out/lzpmc/{v}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if k not in r["Kernel_Name"]: continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(v, json.dumps({a: int(b) for a, b in sorted(agg.items())}))
PY
