"""Build the HIP library in-tree: cartpoleplusplus_amd/libcartpole_hip.so (gfx950).

    python -m cartpoleplusplus_amd.build          # or __graft_entry__.build()
    python -m cartpoleplusplus_amd.build --stamps # + diagnostic phase-stamp build (tools/stamps.py)

hipcc cross-compiles for gfx950 without a GPU.  -ffp-contract=off: only the
explicit __builtin_fmaf calls fuse, which is what makes the kernel agree bit for
bit with the CPU oracle.  -fno-slp-vectorize: the SLP pass packs
independent fp32 FMAs into v_pk_fma_f32 and then pays register-pair moves and
pressure for it (step kernel scratch 324 -> 148 B/lane without it).
The iterative-ILP machine scheduler is measured faster on the step kernel.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
# two translation units, compiled in parallel and linked into one library: the fp32 env
# kernels + raster / event / replay kernels + the C-ABI, and the fp64 env kernels
SRCS = [os.path.join(HERE, "csrc", f) for f in ("cp_kernels.hip", "cp_kernels64.hip")]
DEPS = SRCS + [os.path.join(HERE, "csrc", f) for f in ("cp_common.h", "cp_env.h", "cp_physics.h", "cp_math.h",
                                                     "cp_raster.h", "cp_replay.h")] + [
    os.path.join(HERE, "..", "include", "cartpole_amd.h")]
LIB = os.path.join(HERE, "libcartpole_hip.so")
STAMPS_LIB = os.path.join(HERE, "libcartpole_hip_stamps.so")
ARCH = os.environ.get("CP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

FLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-ffp-contract=off"] + \
        ([] if os.environ.get("CP_SLP") == "1" else ["-fno-slp-vectorize"]) + ["-fPIC",
         "-Wno-unused-result",
         # LLVM's iterative ILP scheduler for gfx9: step kernel 0.634 -> 0.624 ms (r11);
         # scheduling never reorders a rounding, so the results stay bit-identical
         "-mllvm", "-amdgpu-sched-strategy=" + os.environ.get("CP_SCHED_STRATEGY", "iterative-ilp")]


def up_to_date(lib=LIB):
    if not os.path.exists(lib):
        return False
    t = os.path.getmtime(lib)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force=False, verbose=False, stamps=False, variant=None, defines=()):
    """variant: build a diagnostic library libcartpole_hip_<variant>.so with extra -D defines
    (tools/variant_bench.sh runs it through CP_LIB_PATH)."""
    lib = STAMPS_LIB if stamps else LIB
    if variant:
        lib = os.path.join(HERE, f"libcartpole_hip_{variant}.so")
    if not force and up_to_date(lib):
        return lib
    extra = (["-DCP_STAMPS"] if stamps else []) + [f"-D{d}" for d in defines]
    objs, procs = [], []
    for src in SRCS:
        obj = lib + "." + os.path.basename(src) + ".o"
        cmd = [HIPCC] + FLAGS + extra + ["-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
        objs.append(obj)
    for cmd, pr in procs:
        out, _ = pr.communicate()
        if pr.returncode != 0:
            raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + out)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib + ".tmp"] + objs
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc link failed:\n" + res.stdout + res.stderr)
    for o in objs:
        os.remove(o)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    if "--variant" in sys.argv:  # python -m cartpoleplusplus_amd.build --variant TAG DEF1 DEF2 ...
        i = sys.argv.index("--variant")
        print(build(force=True, verbose=True, variant=sys.argv[i + 1], defines=sys.argv[i + 2:]))
        sys.exit(0)
    print(build(force="--force" in sys.argv, verbose=True))
    if "--stamps" in sys.argv:
        print(build(force="--force" in sys.argv, verbose=True, stamps=True))
