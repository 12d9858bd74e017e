set -u
ROUND=r06g TESTS=1 BENCH=0 DIST=1 DIST_ARGS="--train-iters 40 --no-cpu-baseline --no-traffic" bash scripts/gpu_r06.sh || exit $?
REPS=3 LIBS="r05=proud-slam_amd/lib/ab/libpsvo_r05.so cur=" bash scripts/gpu_ab_lib.sh
