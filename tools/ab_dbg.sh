#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in f0 f1 f0 f1; do
  ZCG_LIB=$PWD/variants/$v.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline > gpurun_out/abdbg_$v.json 2>gpurun_out/abdbg_$v.err || { echo "$v failed"; tail -5 gpurun_out/abdbg_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/abdbg_$v.json').read().strip().splitlines()[-1]);print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
