set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
V="abv/base.so abv/pkmin0.so abv/pkmin40.so abv/pkmin64.so abv/pkmin1700.so"
bash tools/ab.sh pkmin/c5w $V -- --envs 2048 --agents 1024 --steps 10 --warmup 2 && \
bash tools/ab.sh pkmin/c3w $V -- --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 && \
bash tools/ab.sh pkmin/c3bots $V -- --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200
