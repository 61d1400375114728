set -u
# A/B of the SLP vectorizer (CP_SLP=1 build: independent fp32 ops packed into v_pk_* instructions)
BENCH_ARGS="--done-on-bounds" bash tools/variant_bench.sh base slp || exit 1
BENCH_ARGS="--continuous" bash tools/variant_bench.sh base slp || exit 1
bash tools/variant_bench.sh base slp || exit 1
for t in base slp; do
  CP_LIB_PATH=$PWD/cartpoleplusplus_amd/libcartpole_hip_$t.so timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'tools'); import host_boundary as h, json; print('$t', json.dumps(h.gym_mirror(steps=1500)))" || exit 1
done
