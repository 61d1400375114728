set -u
mkdir -p gpurun_out
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 300 --warmup 10 --no-cpu-baseline ${ARGS:-} > gpurun_out/ab2_$tag.json 2> gpurun_out/ab2_$tag.err || { echo "$tag failed"; tail -3 gpurun_out/ab2_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab2_$tag.json'));print('$tag', round(d['value']/1e6,2), 'kernel', d['roofline']['avg_launch_ms'], 'reset', d['roofline']['reset_kernel_avg_ms'], 'steady', round(d['steady_state']['value']/1e6,2))"; }
run thr CP_STEP_LATENCY=0 && run lat CP_STEP_LATENCY=1 && run thr2 CP_STEP_LATENCY=0 && run lat2 CP_STEP_LATENCY=1 && run latR CP_STEP_LATENCY=1 CP_RESET_LATENCY=1 && ARGS=--done-on-bounds run bthr CP_STEP_LATENCY=0 && ARGS=--done-on-bounds run blat CP_STEP_LATENCY=1
