set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ZCG_LIB=$PWD/variants/mtf1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bzip2.py -x -q --timeout 300 --timeout-method thread > gpurun_out/bz_mtf_t.log 2>&1 || { tail -20 gpurun_out/bz_mtf_t.log; exit 1; }
for v in mtf0 mtf1; do
  ZCG_LIB=$PWD/variants/$v.so timeout -k 10 300 python -u bench.py --codec bzip2 --steps 3 --warmup 1 --no-extra --no-cpu-baseline > gpurun_out/bz_$v.json 2> gpurun_out/bz_$v.err || exit 1
done
for v in nopipe pipe; do
  ZCG_LIB=$PWD/variants/$v.so timeout -k 10 300 python -u tools/enc_levels.py 512 6,9 > gpurun_out/enc_$v.jsonl 2>&1 || exit 1
done
