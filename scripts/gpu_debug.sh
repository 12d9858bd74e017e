#!/bin/bash
# Short debug pass: staged query path on each golden fixture, then the GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in A_voxels_center B_room0_small; do
  timeout -k 10 120 python scripts/debug_sampler.py $f >> gpurun_out/dbg.log 2>&1
  rc=$?; echo "debug $f rc=$rc"; tail -5 gpurun_out/dbg.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 600 python -m pytest tests -q -x -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
exit $rc
