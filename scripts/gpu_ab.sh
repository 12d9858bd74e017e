#!/bin/bash
# Engine A/B on the GPU box: engine/parity tests, then bench.py headline lines
# with the default build and with each AB_ENV setting ("VAR=value ...", one run each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_gpu_engine.py tests/test_gpu_parity.py}
timeout -k 10 300 python -m pytest $TESTS -q -m gpu -p no:cacheprovider -x > gpurun_out/pytest_ab.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ab.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline > gpurun_out/ab_base.json 2> gpurun_out/ab_base.err
rc=$?; python -c "import json;d=json.load(open('gpurun_out/ab_base.json'));print('base', d['ms_per_step'], d['config']['workload'], d['kernels_ms'])"
[ $rc -ne 0 ] && exit $rc
i=0
for kv in ${AB_ENV:-}; do
  i=$((i+1))
  env $kv timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err
  rc=$?; python -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));print('$kv', d['ms_per_step'], d['kernels_ms'])"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
