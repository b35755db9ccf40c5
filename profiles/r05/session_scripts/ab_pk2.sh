set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pk2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pk2/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -20 gpurun_out/pk2/pytest.log; exit 1; }
tail -2 gpurun_out/pk2/pytest.log
L=gym-macm_amd/libmacm_hip.so
bash tools/ab.sh pk2/c5w abv/base.so $L -- --envs 2048 --agents 1024 --steps 10 --warmup 2 && \
bash tools/ab.sh pk2/big2048 abv/base.so $L -- --envs 256 --agents 2048 --steps 10 --warmup 2 && \
bash tools/ab.sh pk2/tdmbig abv/base.so $L -- --env tdm --teams 1024,1024 --envs 128 --steps 10 --warmup 2 && \
bash tools/ab.sh pk2/c4w abv/base.so $L -- --env tdm --steps 20 --warmup 5 && \
bash tools/ab.sh pk2/c3bots abv/base.so $L -- --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200
