#!/bin/bash
# Inflate A/B session (GPU box): gzip parity subset, variant timings, debug counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TEST_K:-gzip or inflate}" \
  > gpurun_out/pytest_inf.log 2>&1 || { tail -30 gpurun_out/pytest_inf.log; exit 1; }
tail -2 gpurun_out/pytest_inf.log
bash tools/ab_run.sh "--codec gzip" ${VARIANTS:-} || exit 1
timeout -k 10 300 python -u tools/inflate_stats.py 4096 > gpurun_out/inf_stats.json 2>&1 || exit 1
python -c "import json;t=open('gpurun_out/inf_stats.json').read();d=json.loads(t[t.index('{'):]);print(d['cycles_per_round'],d['ms_nodebug'],d['status_ok'],{k:d[k] for k in ('p2h_0_8','p2h_8_16','p2h_16_32','p2h_32_48','p2h_48up','p2_max','rounds')})"
