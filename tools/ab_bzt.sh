#!/bin/bash
# Bzip2 decode A/B, time only: bzip2 GPU tests on the first variant, then
# tools/bz_stats.py (HIP-event time, every chunk checked) per variant.
#   tools/ab_bzt.sh name1 name2 ...   (variants/<name>.so)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
ZCG_LIB=$R/variants/$1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bzip2.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/abbzt_t_$1.log 2>&1 || { echo "variant $1: tests failed"; tail -20 gpurun_out/abbzt_t_$1.log; exit 1; }
tail -1 gpurun_out/abbzt_t_$1.log
for v in "$@"; do
  ZCG_LIB=$R/variants/$v.so timeout -k 10 300 python3 -u tools/bz_stats.py 4096 > gpurun_out/abbzt_$v.json 2>&1 || { echo "stats $v failed"; tail -5 gpurun_out/abbzt_$v.json; exit 1; }
  echo "$v $(tail -c 400 gpurun_out/abbzt_$v.json | tr '\n' ' ')"
done
