#!/bin/bash
# MLP kernel A/B: parity tests, then rocprofv3 kernel stats of mlp_bench for the
# default kernels and for an alternative selected by env (AB_ENV="VAR=value").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_mlp.py tests/test_gpu_engine.py -q -m gpu -p no:cacheprovider -x \
    > gpurun_out/pytest_mlp.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_mlp.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_new -o st -- \
    python3 scripts/mlp_bench.py --iters 20 > gpurun_out/ab_new.log 2>&1
rc=$?; grep fwd+bwd gpurun_out/ab_new.log
[ $rc -ne 0 ] && exit $rc
if [ -n "${AB_ENV:-}" ]; then
  export ${AB_ENV}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_old -o st -- \
      python3 scripts/mlp_bench.py --iters 20 > gpurun_out/ab_old.log 2>&1
  rc=$?; grep fwd+bwd gpurun_out/ab_old.log
fi
exit $rc
