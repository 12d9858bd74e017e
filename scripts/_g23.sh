set -u
ROUND=r06t TESTS=1 BENCH=1 PROFILE=1 CONFIGS=0 DIST=1 DIST_ARGS="--train-iters 40 --no-cpu-baseline --no-traffic" STEPS=20 TL_ITERS="-30 -25" bash scripts/gpu_r06.sh
