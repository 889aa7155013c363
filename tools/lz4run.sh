set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "lz4 or c1 or parity or abi" --timeout 300 --timeout-method thread > gpurun_out/pytest_lz4.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_lz4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --codec lz4 --steps 3 --warmup 1 --no-extra --no-cpu-baseline > gpurun_out/bench_lz4.json 2>gpurun_out/bench_lz4.err
rc=$?
cat gpurun_out/bench_lz4.json; tail -3 gpurun_out/bench_lz4.err
exit $rc
