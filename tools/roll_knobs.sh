# rollout A/B of wave-kernel knobs (ab/v*.so): M window, M steady, C4 window
set -u
mkdir -p gpurun_out/knobs
for v in v0 v1 v2 v3; do
  MACM_LIB=ab/$v.so timeout -k 10 120 python -u tools/rollout_ab.py > gpurun_out/knobs/m_win_$v.json 2> gpurun_out/knobs/m_win_$v.err || exit 1
  MACM_LIB=ab/$v.so timeout -k 10 120 python -u tools/rollout_ab.py --warmup 100 --steps 200 > gpurun_out/knobs/m_ss_$v.json 2> gpurun_out/knobs/m_ss_$v.err || exit 1
  MACM_LIB=ab/$v.so timeout -k 10 120 python -u tools/rollout_ab.py --env tdm > gpurun_out/knobs/c4_win_$v.json 2> gpurun_out/knobs/c4_win_$v.err || exit 1
done
