set -uo pipefail
mkdir -p gpurun_out/shape_win
for rep in 1 2; do for s in throughput latency; do
timeout -k 10 150 python bench.py --no-cpu-baseline --no-steady-state --no-median --shape $s --steps 20 --warmup 5 > gpurun_out/shape_win/w_${s}_$rep.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/shape_win/w_${s}_$rep.json'));print('win $s', round(d['value']/1e6,2), d['roofline']['avg_launch_ms'])"
timeout -k 10 150 python bench.py --no-cpu-baseline --no-steady-state --no-median --shape $s --steps 200 --warmup 5 > gpurun_out/shape_win/c_${s}_$rep.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/shape_win/c_${s}_$rep.json'));print('200 $s', round(d['value']/1e6,2), d['roofline']['avg_launch_ms'])"
done; done
