set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
V="abv/cur.so abv/noprio.so abv/lanedum.so"
bash tools/ab.sh bknobs/c5w $V -- --envs 2048 --agents 1024 --steps 10 --warmup 2 && \
bash tools/ab.sh bknobs/c3w $V -- --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5
