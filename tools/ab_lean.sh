set -u
bash tools/gpu_tests.sh rd5g || exit 1
BENCH_ARGS="--done-on-bounds" bash tools/variant_bench.sh base lean all || exit 1
BENCH_ARGS="--continuous" bash tools/variant_bench.sh base all || exit 1
for t in base all; do
  CP_LIB_PATH=$PWD/cartpoleplusplus_amd/libcartpole_hip_$t.so timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'tools'); import host_boundary as h, json; print('$t', json.dumps(h.gym_mirror(steps=1500)))" || exit 1
done
