#!/bin/bash
# File -> host rate of the native store (tools/e2e_store.py) for gzip, raw and lz4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/e2e_store.jsonl
for c in raw gzip lz4; do
  timeout -k 10 300 python -u tools/e2e_store.py --codec $c --chunks 2048 >> gpurun_out/e2e_store.jsonl 2> gpurun_out/e2e_$c.err || { echo "e2e $c failed"; tail -5 gpurun_out/e2e_$c.err; exit 1; }
done
cat gpurun_out/e2e_store.jsonl
