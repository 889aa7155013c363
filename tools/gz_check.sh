set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gzip or inflate or c1 or golden or zarrita" > gpurun_out/pytest_gz.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gz.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/pytest_gz.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/iw_stats.py 4096 > gpurun_out/iw_stats.json 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --codec gzip --steps 5 --warmup 1 --no-extra --no-cpu-baseline > gpurun_out/bg.json 2>&1 || exit 1
python3 -c "
import json;d=json.loads(open('gpurun_out/iw_stats.json').read()[open('gpurun_out/iw_stats.json').read().index('{'):])
print({k:d[k] for k in ('wave_ms_med','wave_bad_chunks','wave_status_ok','blockpar_ms_med')}); print(d['cycle_share']); print(d['kcyc_per_chunk_total'])
r=json.loads(open('gpurun_out/bg.json').read().strip().splitlines()[-1]); print('bench', r['value'], r['ms_per_step'])"
