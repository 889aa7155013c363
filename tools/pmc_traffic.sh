#!/bin/bash
# HBM traffic per launch of every bench leg (GPU box), measured on the SAME
# bench code, streams and batch sizes that bench.py reports.
# One rocprofv3 --pmc pass per counter group (FETCH_SIZE takes 3 of the 4
# TCC slots, WRITE_SIZE 2, so they cannot share a pass; the third pass holds
# the sized read requests TCC_EA0_RDREQ_{32,64,128}B, which check the
# calibration's 128 B request assumption on the leg itself), each under its
# own time limit; the first failure ends the script.
#   usage: tools/pmc_traffic.sh OUTDIR [leg ...]   (legs: gzip lz4 raw xz bzip2 {gzip,lz4,xz,bzip2}_encode)
set -o pipefail
out=$(realpath -m "$1"); shift
legs=${*:-gzip lz4 raw xz bzip2 gzip_encode lz4_encode xz_encode bzip2_encode}
root="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for c in $legs; do
  case $c in
    *_encode) args="--codec raw --batch 1 --steps 2 --warmup 1 --legs $c --no-cpu-baseline";;
    *) args="--codec $c --steps 2 --warmup 1 --no-extra --no-cpu-baseline";;
  esac
  for k in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B"; do
    d=${k%% *}; [ "$d" = TCC_EA0_RDREQ ] && d=RDREQ
    timeout -s KILL 300 rocprofv3 --pmc $k --output-format csv -d "$out/$c.$d" -o pmc -- \
      python3 "$root/bench.py" $args > "$out/$c.$d.log" 2>&1 || exit $?
  done
done
