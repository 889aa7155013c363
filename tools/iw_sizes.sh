#!/bin/bash
# Wave-per-chunk vs 256-lane inflate kernel time across batch sizes
# (tools/iw_stats.py per size).  Usage: tools/iw_sizes.sh 256 1024 4096
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in "$@"; do
  timeout -k 10 300 python -u tools/iw_stats.py "$n" > gpurun_out/iwsz_$n.json 2>&1 || { echo "n=$n failed"; tail -5 gpurun_out/iwsz_$n.json; exit 1; }
  python3 - "$n" <<'PY'
import json, sys
t = open(f"gpurun_out/iwsz_{sys.argv[1]}.json").read(); d = json.loads(t[t.index("{"):])
print("n", sys.argv[1], "wave_ms", d["wave_ms_med"], "par_ms", d["blockpar_ms_med"], "bad", d["wave_bad_chunks"], d["blockpar_bad_chunks"])
PY
done
