#!/bin/bash
# A/B timing of library variants on the GPU box: for each variants/<name>.so
# run the bench's main leg with ZCG_LIB pointing at it.
#   tools/ab_run.sh "<bench args>" name1 name2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ARGS=$1; shift
for v in "$@"; do
  ZCG_LIB=$PWD/variants/$v.so timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline $ARGS \
    > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "variant $v failed rc=$?"; exit 1; }
  python - "$v" <<'PY'
import json,sys
r=json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], r["value"], r["unit"], r["ms_per_step"], "ms/step")
PY
done
