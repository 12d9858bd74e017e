#!/bin/bash
# Round-4 GPU session: selected GPU tests (TESTS, default the whole -m gpu
# suite), then optionally a same-box A/B of library builds / switches
# (LIBS, scripts/gpu_ab_lib.sh).  Each GPU step has its own time limit; the
# script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04}
if [ "${TESTS:-all}" != "none" ]; then
  T=${TESTS:-tests}
  [ "$T" = "all" ] && T=tests
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $T -x -v -m gpu -p no:cacheprovider --timeout 300 \
      --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/${R}_pytest.log | tail -5
  [ $rc -ne 0 ] && { tail -60 gpurun_out/${R}_pytest.log; exit $rc; }
fi
if [ -n "${LIBS:-}" ]; then
  bash scripts/gpu_ab_lib.sh || exit $?
fi
echo done
