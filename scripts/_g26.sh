set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for sc in scannet0000 multiroom; do
  timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06v_$sc -o run -- \
      python3 bench.py --scene $sc --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --train-iters 100 > gpurun_out/r06v_${sc}_bench.json 2> gpurun_out/r06v_$sc.err
  echo "$sc rc=$?"
  python3 scripts/ba_timeline.py gpurun_out/r06v_$sc/run_kernel_trace.csv -- -10 > gpurun_out/r06v_${sc}_timeline.txt 2>&1 || true
  rm -f gpurun_out/r06v_$sc/run_agent_info.csv
done
