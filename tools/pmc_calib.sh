#!/bin/bash
# Counter calibration passes (GPU box): tools/probe/pmc_calib (prebuilt) under
# one rocprofv3 --pmc pass per counter group, each under its own time limit;
# the first failure ends the script.  Reduce with tools/pmc_calib.py.
#   usage: tools/pmc_calib.sh OUTDIR [log2 buffer bytes]
set -o pipefail
out=$(realpath -m "$1")
lg=${2:-30}
root="${GRAFT_REPO_ROOT:-/root/repo}"
bin="$root/tools/probe/pmc_calib"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 "$bin" "$lg" > "$out/plain.jsonl" 2> "$out/plain.err" || exit $?
timeout -s KILL 60 rocprofv3 -L > "$out/avail.txt" 2>&1 || true
timeout -k 10 300 "$bin" 33 > "$out/plain33.jsonl" 2> "$out/plain33.err" || exit $?
# one pass per counter group (<= 4 TCC counters a pass; FETCH_SIZE takes 3, WRITE_SIZE 2)
for k in FETCH_SIZE WRITE_SIZE \
         "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" \
         "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B" "TCC_EA0_RDREQ_DRAM TCC_EA0_RDREQ_DRAM_32B" "TCC_HIT TCC_MISS"; do
  d=${k// /+}
  timeout -s KILL 120 rocprofv3 --pmc $k --output-format csv -d "$out/$d" -o pmc -- \
    "$bin" "$lg" > "$out/$d.jsonl" 2> "$out/$d.err" || exit $?
done
