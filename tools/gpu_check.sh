#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-5}
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err \
 && cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
rc=$?
echo "exit=$rc"
tail -5 "$GRAFT_REPO_ROOT/gpurun_out/pytest_gpu.log"
cat "$GRAFT_REPO_ROOT/gpurun_out/bench.json" 2>/dev/null
exit $rc
