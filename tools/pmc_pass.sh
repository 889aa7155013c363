#!/bin/bash
# One rocprofv3 PMC pass per counter group over a short command (GPU box).
# usage: tools/pmc_pass.sh OUTDIR "CNT1 CNT2 ..." -- python3 bench.py ...
set -o pipefail
out=$1; shift; cnts=$1; shift; shift
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $cnts -d "$out" -o pmc --output-format csv -- "$@" > "$out.log" 2>&1
