#!/bin/bash
# round 4: per-call host profile of bundle_adjust_frames (K = 20), and the
# W = 256 decoder kernels alone at config C's sample count (rocprofv3 stats)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04l}
PSVO_BA_PROFILE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic \
    > gpurun_out/${R}_callprof.json 2> gpurun_out/${R}_callprof.err || exit $?
grep "ba-call" gpurun_out/${R}_callprof.err | tail -4
python3 -c "import json;d=json.load(open('gpurun_out/${R}_callprof.json'));print(d['ms_per_step'], d['gpu_ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_m256 -o m -- \
    python3 scripts/mlp_bench.py --width 256 --m 466287 --iters 10 > gpurun_out/${R}_m256.log 2>&1
rc=$?; echo "m256 rc=$rc"; tail -1 gpurun_out/${R}_m256.log; [ $rc -ne 0 ] && exit $rc
python3 scripts/prof_summary.py gpurun_out/${R}_m256/m_kernel_stats.csv 8
echo done
