#!/bin/bash
# LZ4 lane decoder A/B: parity tests of the lane paths on each variant, then
# the C4 leg at 8 192 (one GPU's share of C4 at 8 GPUs) and 65 536 chunks.
#   tools/ab_lz4q.sh name1 name2 ...   (variants/<name>.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in "$@"; do
  ZCG_LIB=$PWD/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4_paths.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_t_$v.log 2>&1 \
    || { echo "variant $v: tests failed"; tail -20 gpurun_out/ab_t_$v.log; exit 1; }
  for b in 8192 65536; do
    ZCG_LIB=$PWD/variants/$v.so timeout -k 10 300 python -u bench.py --codec lz4 --global-batch $b --steps 3 --warmup 1 --no-extra --no-cpu-baseline \
      > gpurun_out/ab_${v}_$b.json 2> gpurun_out/ab_${v}_$b.err || { echo "variant $v b=$b failed"; tail -5 gpurun_out/ab_${v}_$b.err; exit 1; }
    python3 - "$v" "$b" <<'PY'
import json,sys
r=json.loads(open(f"gpurun_out/ab_{sys.argv[1]}_{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], sys.argv[2], r["value"], r["unit"], r["ms_per_step"], "ms/step", r["roofline"].get("kernel"), r["roofline"].get("kernel_ms"))
PY
  done
done
