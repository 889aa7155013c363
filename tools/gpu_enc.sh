#!/bin/bash
# Gzip encode (zlib-exact path) + LZ4 decode GPU tests, then a kernel profile of
# the bench's gzip_encode leg.  usage: tools/gpu_enc.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-enc}
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_lz4_paths.py -x -q --timeout 300 \
  --timeout-method thread -k "gzip or lz4" > gpurun_out/${tag}_t.log 2>&1 || { tail -30 gpurun_out/${tag}_t.log; exit 1; }
tail -1 gpurun_out/${tag}_t.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$tag" -o enc -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --legs gzip_encode --no-cpu-baseline \
  > "$GRAFT_REPO_ROOT/gpurun_out/${tag}_bench.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/${tag}_bench.log"; exit 1; }
tail -1 "$GRAFT_REPO_ROOT/gpurun_out/${tag}_bench.log"
