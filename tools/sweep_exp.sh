set -e
for it in 1 10 25 50; do
  timeout -k 10 300 python bench.py --steps 300 --warmup 10 --no-cpu-baseline --solver-iterations $it > gpurun_out/exp_it$it.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/exp_it$it.json'));print($it, d['value'], d['roofline']['avg_launch_ms'], d['roofline']['reset_kernel_avg_ms'])"
done
