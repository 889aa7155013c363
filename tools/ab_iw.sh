#!/bin/bash
# Inflate (wave per chunk) A/B: gzip parity tests, then tools/iw_stats.py
# (HIP-event time, all chunks checked, phase counters) per variant.
#   tools/ab_iw.sh name1 name2 ...   (variants/<name>.so; build them with
#   -DZIW_DBG=1 for the phase cycle shares: the product build compiles the
#   debug counters out and reports zero shares)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  export ZCG_LIB=$PWD/variants/$v.so
  if [ -z "$NO_TESTS" ]; then
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gzip or inflate or c1 or golden" \
      > gpurun_out/abiw_t_$v.log 2>&1 || { echo "variant $v: tests failed"; tail -30 gpurun_out/abiw_t_$v.log; exit 1; }
  fi
  timeout -k 10 300 python -u tools/iw_stats.py 4096 > gpurun_out/abiw_$v.json 2>&1 || { echo "variant $v: stats failed"; tail -5 gpurun_out/abiw_$v.json; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
t = open(f"gpurun_out/abiw_{sys.argv[1]}.json").read(); d = json.loads(t[t.index("{"):])
print(sys.argv[1], "ms", d["wave_ms_med"], "bad", d["wave_bad_chunks"], "ok", d["wave_status_ok"], "kcyc/chunk", d["kcyc_per_chunk_total"], json.dumps(d["cycle_share"]))
PY
done
