set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
V="abv/cur.so abv/noprio.so"
bash tools/ab.sh bknobs2/c3bots $V -- --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200 && \
bash tools/ab.sh bknobs2/c3w $V -- --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 && \
bash tools/ab.sh bknobs2/c5w $V -- --envs 2048 --agents 1024 --steps 10 --warmup 2 && \
bash tools/ab.sh bknobs2/big2048 $V -- --envs 256 --agents 2048 --steps 10 --warmup 2
