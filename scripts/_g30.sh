set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/r06z_tl -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/r06z_tl_bench.json 2> gpurun_out/r06z_tl.err
echo "rc=$?"
python3 scripts/ba_timeline.py gpurun_out/r06z_tl/run_kernel_trace.csv -- -10 > gpurun_out/r06z_timeline.txt 2>&1 || true
python3 scripts/launch_gaps.py gpurun_out/r06z_tl 10 > gpurun_out/r06z_gaps.txt 2>&1 || true
rm -f gpurun_out/r06z_tl/run_agent_info.csv gpurun_out/r06z_tl/run_hip_api_trace.csv
