#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the call.
#   env: PYTEST_ARGS (extra pytest args), STEPS, SKIP_TESTS=1, SKIP_PROF=1, BENCH_ARGS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-5}
run_tests() {
  [ -n "$SKIP_TESTS" ] && return 0
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
    > gpurun_out/pytest_gpu.log 2>&1 \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
}
run_bench() {
  timeout -k 10 900 python -u bench.py --steps $STEPS --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
}
run_prof() {
  [ -n "$SKIP_PROF" ] && return 0
  cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$R/gpurun_out/prof.log" 2>&1 && grep "^{" "$R/gpurun_out/prof.log" > "$R/gpurun_out/prof_bench.json"
}
run_tests && run_bench && run_prof
rc=$?
echo "exit=$rc"
tail -5 "$R/gpurun_out/pytest_gpu.log" 2>/dev/null
cat "$R/gpurun_out/bench.json" 2>/dev/null
exit $rc
