#!/bin/bash
# Instruction-cache counters of the inflate kernel on the C2 bench batch
# (one rocprofv3 --pmc pass per set).  usage: tools/iw_icache.sh [variant]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
[ -n "$1" ] && export ZCG_LIB=$R/variants/$1.so
tag=${1:-base}
mkdir -p "$R/gpurun_out/icache_$tag"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVES" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/icache_$tag/p$i" -o pmc -- \
    python3 "$R/tools/iw_stats.py" 4096 > "$R/gpurun_out/icache_$tag/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/icache_$tag/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_sum.py" $(ls "$R"/gpurun_out/icache_$tag/p*/*counter_collection.csv "$R"/gpurun_out/icache_$tag/p*/*/*counter_collection.csv 2>/dev/null) | grep -A1 inflate_wave
