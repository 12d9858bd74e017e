set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=3 LIBS="cur= gmark=proud-slam_amd/lib/ab/libpsvo_gmark.so" bash scripts/gpu_ab_lib.sh || exit $?
echo "== E with PMC traffic"
timeout -k 10 600 python bench.py --scene multiroom --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06p_bench_E.json 2> gpurun_out/r06p_bench_E.err; rc=$?
echo "E rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 -c "
import json;d=json.loads(open('gpurun_out/r06p_bench_E.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['value'], d['ms_per_step'], r['frac'], r['frac_hbm_counters'], r['traffic'], {k:(v['ms'], v.get('frac_hbm_counters')) for k,v in r['per_region'].items()})"
