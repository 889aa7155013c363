#!/bin/bash
# Bzip2 decode A/B: the in-tree library ("prod") and variants/<name>.so:
# tools/bz_stats.py timers + time on the bench-shaped batch, then FETCH/WRITE
# of the bzip2 bench leg per build.   usage: tools/ab_bz.sh name1 ...
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
for v in prod "$@"; do
  if [ "$v" = prod ]; then lib="$R/zarr_amd/libzchunk_gpu.so"; else lib="$R/variants/$v.so"; fi
  ZCG_LIB=$lib timeout -k 10 300 python3 -u tools/bz_stats.py 4096 > gpurun_out/abbz_$v.json 2>&1 || { echo "stats $v failed"; tail -5 gpurun_out/abbz_$v.json; exit 1; }
  echo "$v $(tail -c 600 gpurun_out/abbz_$v.json | tr '\n' ' ')"
  rm -rf "$R/gpurun_out/bzpmc_$v"
  ZCG_LIB=$lib tools/pmc_traffic.sh "$R/gpurun_out/bzpmc_$v" bzip2 || { echo "pmc $v failed"; exit 1; }
  python3 tools/pmc_traffic.py "gpurun_out/bzpmc_$v" "gpurun_out/bzpmc_$v.json" > /dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['legs']['bzip2']; print(sys.argv[2], 'fetch GB', d['fetch_bytes']/1e9, 'write GB', d['write_bytes']/1e9)" "gpurun_out/bzpmc_$v.json" "$v"
done
