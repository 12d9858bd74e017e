#!/bin/bash
# One iteration on k_mlp_bwd3: decoder tests, phase stamps, a short bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-b3}
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_mlp.py} -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/mlp_stamps.py ${M:-261107} > gpurun_out/${T}_stamps.txt 2>&1
rc=$?; grep -A9 bwd3 gpurun_out/${T}_stamps.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; [ $rc -ne 0 ] && exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/${T}_bench.json'));print('ms/step', round(d['ms_per_step'],4), {k: round(v*1e3,1) for k,v in d['kernels_ms_overlapped'].items()})"
