set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in cur r05; do
  lib=proud-slam_amd/lib/diag/libpsvo_is_stamps.so; [ $v = r05 ] && lib=proud-slam_amd/lib/diag/libpsvo_is_stamps_r05.so
  PSVO_DIAG_LIB=$lib timeout -k 10 300 python scripts/intersect_stamps.py multiroom > gpurun_out/r06l_is_stamps_E_$v.txt 2>&1 || { echo "is_stamps $v failed"; tail -5 gpurun_out/r06l_is_stamps_E_$v.txt; exit 1; }
  echo "== E traversal stamps $v"; grep -v amdgpu.ids gpurun_out/r06l_is_stamps_E_$v.txt | tail -6
  PSVO_DIAG_LIB=$lib timeout -k 10 300 python scripts/sampler_stamps.py --train-iters 0 > gpurun_out/r06l_smp_stamps_$v.txt 2>&1 || { echo "smp_stamps $v failed"; tail -5 gpurun_out/r06l_smp_stamps_$v.txt; exit 1; }
  echo "== B sampler stamps $v"; grep -A20 "k_sample_fused" gpurun_out/r06l_smp_stamps_$v.txt | head -16
done
REPS=2 STEPS=20 BENCH_ARGS="--scene multiroom --train-iters 0" LIBS="r05E=proud-slam_amd/lib/ab/libpsvo_r05.so curE=" bash scripts/gpu_ab_lib.sh || exit $?
