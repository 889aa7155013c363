#!/bin/bash
# HBM traffic per decode launch for every codec's bench leg (GPU box).
# One rocprofv3 --pmc pass per counter (FETCH_SIZE takes 3 of the 4 TCC
# slots, WRITE_SIZE 2, so they cannot share a pass), each under its own
# time limit; the first failure ends the script.
#   usage: tools/pmc_traffic.sh OUTDIR [codec ...]
set -o pipefail
out=$1; shift
codecs=${*:-gzip lz4 raw xz bzip2}
root="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for c in $codecs; do
  case $c in
    lz4) b=4096;; xz|bzip2) b=2048;; raw) b=1024;; *) b=4096;;
  esac
  for k in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $k --output-format csv -d "$out/$c.$k" -o pmc -- \
      python3 "$root/bench.py" --codec $c --batch $b --steps 2 --warmup 1 --no-extra --no-cpu-baseline \
      > "$out/$c.$k.log" 2>&1 || exit $?
  done
done
