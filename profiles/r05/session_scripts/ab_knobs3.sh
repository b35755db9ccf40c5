set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
V="abv/cur.so abv/noislp.so"
bash tools/ab.sh knobs3/c3w $V -- --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 && \
bash tools/ab.sh knobs3/c3bots $V -- --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200 && \
bash tools/ab.sh knobs3/c5w $V -- --envs 2048 --agents 1024 --steps 10 --warmup 2 && \
bash tools/env_ab.sh knobs3/slices_c3 MACM_WG_SLICES "2 3 4" --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5
