set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=4 LIBS="cur= smpnohelp=proud-slam_amd/lib/ab/libpsvo_smpnohelp.so r05=proud-slam_amd/lib/ab/libpsvo_r05.so" bash scripts/gpu_ab_lib.sh || exit $?
