#!/bin/bash
# Encoder A/B: gzip encode tests, then tools/enc_stats.py (time, ratio, stream hashes) per variant.
#   tools/ab_enc.sh codec name1 name2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
C=$1; shift
for v in "$@"; do
  export ZCG_LIB=$PWD/variants/$v.so
  timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py -x -q --timeout 300 --timeout-method thread -k "$C" \
    > gpurun_out/abenc_t_$v.log 2>&1 || { echo "variant $v: tests failed"; tail -30 gpurun_out/abenc_t_$v.log; exit 1; }
  tail -1 gpurun_out/abenc_t_$v.log
  timeout -k 10 300 python -u tools/enc_stats.py 512 $C > gpurun_out/abenc_$v.json 2>&1 || { echo "variant $v: stats failed"; tail -5 gpurun_out/abenc_$v.json; exit 1; }
  echo "== $v"; grep -v "^$" gpurun_out/abenc_$v.json | grep -v amdgpu.ids
done
