#!/bin/bash
# The pinned e2e table of DESIGN §7 in one GPU call: decode and encode
# directions of tools/e2e_bench.py, then the store path (tools/e2e_store.py),
# one JSON line each -> gpurun_out/e2e_all.jsonl.  Every step has its own
# time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/e2e_all.jsonl
: > "$out"
run() {
  timeout -k 10 240 python -u "$@" >> "$out" 2> gpurun_out/e2e_all.err || { echo "failed: $*"; tail -5 gpurun_out/e2e_all.err; exit 1; }
}
run tools/e2e_bench.py --codec gzip --chunks 3072 --sub 768 --streams 2
run tools/e2e_bench.py --codec gzip --chunks 1024 --sub 256 --streams 2
run tools/e2e_bench.py --codec lz4 --chunks 8192 --sub 4096 --streams 2
run tools/e2e_bench.py --codec raw --chunks 1024 --sub 256 --streams 2
run tools/e2e_bench.py --codec xz --chunks 4096 --sub 2048 --streams 2
run tools/e2e_bench.py --codec bzip2 --chunks 4096 --sub 2048 --streams 2
run tools/e2e_bench.py --encode --codec gzip --chunks 1024 --sub 256 --streams 2
run tools/e2e_bench.py --encode --codec lz4 --chunks 1024 --sub 256 --streams 2
run tools/e2e_bench.py --encode --codec xz --chunks 1024 --sub 256 --streams 2
run tools/e2e_bench.py --encode --codec bzip2 --chunks 1024 --sub 256 --streams 2
for c in raw gzip lz4; do run tools/e2e_store.py --codec $c --chunks 2048; done
cat "$out"
