#!/bin/bash
# round 4: chain-variant tests, A/B of the chain variants, a per-call host profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_engine_fullsize_grads.py -x -v -m gpu \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04e_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r04e_pytest.log | tail -3
[ $rc -ne 0 ] && { tail -40 gpurun_out/r04e_pytest.log; exit $rc; }
PSVO_BA_PROFILE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic \
    > gpurun_out/r04e_callprof.json 2> gpurun_out/r04e_callprof.err || exit $?
grep "ba-call" gpurun_out/r04e_callprof.err | tail -4
REPS=3 STEPS=60 LIBS="base=proud-slam_amd/lib/ab/libpsvo_base.so new= padded=PSVO_PADDED_Z=1 rays=PSVO_INTERP_RAYS=1 dev=PSVO_DEV_SIZED=1" \
    bash scripts/gpu_ab_lib.sh || exit $?
echo done
