"""Every diagnostic compile-time switch of the kernels still compiles (the A/B variants that
DESIGN.md §5 measured and did not adopt must not bit-rot in the product headers).  Each switch is
checked with hipcc's device-side semantic analysis (-fsyntax-only: every kernel template the launchers
reference is instantiated, no code generation), for both translation units (fp32 cp_kernels.hip and
fp64 cp_kernels64.hip).  CPU only; a few seconds per check, run in parallel."""
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cartpoleplusplus_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# diagnostic switches (DESIGN.md §5 and the comments at their definitions); "" = the product build
SWITCHES = ["", "CP_STAMPS", "CP_STAMPS CP_STAMP_C44", "CP_P1", "CP_P1 CP_P1_CHECK=1", "CP_STEP_C44=1",
            "CP_CROSS_OPAQUE=1", "CP_PRIO_MERGED", "CP_PRIO_MODE=1", "CP_PRIO_MODE=2", "CP_PRIO_AFTER=0",
            "CP_DIAG_NO_CROSS", "CP_UNROLL_ROWS=1", "CP_HDR_SCRATCH", "CP_NO_GROUND_PEEL", "CP_NO_EZ", "CP_NO_C4K",
            "CP_NO_C44", "CP_NO_FAST_ROWS", "CP_NO_NONFINITE", "CP_NT_OUT", "CP_SOA_AUX=2", "CP_ALLIN_STEP=0",
            "CP_C44_CHECK=1", "CP_WAVES_PER_EU=1", "CP_RV_NO_DENSE", "CP_RV_NO_OUTPUT", "CP_RV_NO_STORE",
            "CP_RV_SPT=3", "CP_RV_STOP=0", "CP_RV_STOP=1", "CP_NO_LEAN_C4", "CP_NO_LEAN_STEP", "CP_LEAN_TP", "CP_NO_HC2", "CP_NO_EDGE_SKIP", "CP_STAMPS CP_STAMP_BB", "CP_HX_TP", "CP_NO_LATE_I", "CP_NO_LATE_G", "CP_NO_LEAN_TR", "CP_LEAN_F64", "CP_NO_WSM", "CP_NO_LATE_ISL", "CP_NO_LATE_BAX"]


def _check(defs, tu):
    cmd = [HIPCC, "--offload-arch=gfx950", "-std=c++17", "--cuda-device-only", "-fsyntax-only",
           *[f"-D{d}" for d in defs.split()], os.path.join(CSRC, tu)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    return defs, tu, r.returncode, r.stderr[-3000:]


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_every_diagnostic_switch_compiles():
    jobs = [(d, tu) for d in SWITCHES for tu in ("cp_kernels.hip", "cp_kernels64.hip")]
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = list(ex.map(lambda j: _check(*j), jobs))
    bad = [(d, tu, err) for d, tu, rc, err in res if rc != 0]
    assert not bad, "\n".join(f"-D{d} {tu}:\n{err}" for d, tu, err in bad[:3])
