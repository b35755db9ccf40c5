set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/ab.sh unroll4/c5w abv/cur.so abv/unroll4.so -- --envs 2048 --agents 1024 --steps 10 --warmup 2 && \
bash tools/ab.sh unroll4/c3w abv/cur.so abv/unroll4.so -- --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 && \
bash tools/ab.sh unroll4/c3bots abv/cur.so abv/unroll4.so -- --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200
