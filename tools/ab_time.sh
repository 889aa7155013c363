#!/bin/bash
# Timing-only A/B of LZ4 decode variants (no parity: diagnostic builds).
#   tools/ab_time.sh n name1 name2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
N=$1; shift
for v in "$@"; do
  ZCG_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u tools/lz4_time.py $N || { echo "variant $v failed"; exit 1; }
done
