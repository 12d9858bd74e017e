set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in gate nogate; do
  g=1; [ $mode = nogate ] && g=0
  PSVO_BA_DRAW_GATE=$g timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/r06s_$mode -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --train-iters 100 > gpurun_out/r06s_${mode}_bench.json 2> gpurun_out/r06s_$mode.err
  echo "$mode rc=$?"
  python3 scripts/ba_timeline.py gpurun_out/r06s_$mode/run_kernel_trace.csv -- -10 > gpurun_out/r06s_${mode}_timeline.txt 2>&1 || true
  rm -f gpurun_out/r06s_$mode/run_agent_info.csv
done
