set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
python tools/lz4_stats.py 8192
