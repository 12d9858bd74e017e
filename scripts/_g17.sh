set -u
# full GPU suite + default bench (trained, PMC traffic) + rocprof kernel trace / timelines + configs C and E
ROUND=r06n TESTS=1 BENCH=1 PROFILE=1 CONFIGS=1 STEPS=20 TL_ITERS="-30 -25" bash scripts/gpu_r06.sh
