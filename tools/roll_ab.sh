# per-step launches vs one rollout launch (tools/rollout_ab.py), product library
set -u
mkdir -p gpurun_out/roll
r() { local n=$1; shift; timeout -k 10 120 python -u tools/rollout_ab.py "$@" > gpurun_out/roll/$n.json 2> gpurun_out/roll/$n.err || exit 1; }
r m_win
r m_ss --warmup 100 --steps 100
r c4_win --env tdm
r c4_ss --env tdm --warmup 100 --steps 100
r c2_ss --envs 1024 --warmup 100 --steps 100
r m_1000 --warmup 100 --steps 1000 --reps 2
