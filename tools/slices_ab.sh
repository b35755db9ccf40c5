set -u
mkdir -p gpurun_out/sl
for s in 1 2 3 4; do
  MACM_SLICES=$s MACM_LIB=ab/slices.so timeout -k 10 150 python -u tools/rollout_ab.py --agents 256 --flocks 4 --reps 2 > gpurun_out/sl/c3_$s.json 2> gpurun_out/sl/c3_$s.err || exit 1
done
