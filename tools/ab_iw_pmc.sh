#!/bin/bash
# HBM traffic of the gzip bench leg per inflate variant (variants/<name>.so):
#   tools/ab_iw_pmc.sh name1 name2 ...  -> gpurun_out/iwpmc_<name>.json
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
for v in "$@"; do
  rm -rf "$R/gpurun_out/iwpmc_$v"
  ZCG_LIB="$R/variants/$v.so" "$R/tools/pmc_traffic.sh" "$R/gpurun_out/iwpmc_$v" gzip || { echo "pmc $v failed"; exit 1; }
  (cd "$R" && python3 tools/pmc_traffic.py "gpurun_out/iwpmc_$v" "gpurun_out/iwpmc_$v.json" > /dev/null) || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['legs']['gzip']; print(sys.argv[2], 'fetch GB', d['fetch_bytes']/1e9, 'write GB', d['write_bytes']/1e9)" "$R/gpurun_out/iwpmc_$v.json" "$v"
done
