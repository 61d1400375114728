"""bench.py's C5 roofline names the render kernel the library itself launches (cp_render_kernel_name,
ADVICE r4): no re-derivation of launch_render's LDS layout in Python."""
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_asks_the_library_for_the_render_kernel():
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "env.render_kernel_name()" in src
    assert not hasattr(bench, "SMALL2_PAIRS") and not hasattr(bench, "render_kernel_name")


def _summary(tmp_path, name, workload, hbm=123456, valu=789):
    import json
    d = {"tag": name, "kernels": {"cp_step_kernel<discrete>": {"hbm_bytes_per_launch": hbm,
                                                              "sq_per_launch": {"SQ_INSTS_VALU": valu}}}}
    if workload is not None:
        d["workload"] = workload
    p = tmp_path / f"{name}_pmc.json"
    p.write_text(json.dumps(d))
    return str(p)


WANT = {"batch": 65536, "repeats": 3, "action_kind": "discrete", "dtype": "f32", "step_shape": "throughput",
        "lib_sha256": "ab" * 32}


def test_pmc_summary_must_match_workload_and_library(tmp_path):
    """roofline.traffic and valu come only from a PMC summary collected on the timed workload with the
    library the bench loaded: a summary of another build, or one without the keys,
    gives traffic None with a reason."""
    other = dict(WANT, lib_sha256="cd" * 32)
    files = [_summary(tmp_path, "z_other_build", other), _summary(tmp_path, "y_keyless", None)]
    for f in (bench.pmc_traffic, bench.pmc_valu):
        v, src, why = f("cp_step_kernel<discrete>", WANT, files)
        assert v is None and src is None
        assert "lib_sha256" in why and "no workload keys" in why, why
    partial = {k: v for k, v in WANT.items() if k != "dtype"}
    v, _, why = bench.pmc_traffic("cp_step_kernel<discrete>", WANT, [_summary(tmp_path, "x_partial", partial)])
    assert v is None and "'dtype'" in why
    good = _summary(tmp_path, "a_good", dict(WANT), hbm=42, valu=7)
    v, src, why = bench.pmc_traffic("cp_step_kernel<discrete>", WANT, files + [good])
    assert v == 42 and src.endswith("a_good_pmc.json") and why is None
    assert bench.pmc_valu("cp_step_kernel<discrete>", WANT, files + [good])[0] == 7
    v, _, why = bench.pmc_traffic("cp_step_kernel<continuous>", WANT, files)
    assert v is None and "holds" in why


def test_summarizer_records_the_workload_keys(tmp_path):
    """tools/summarize_profile.py writes every bench.PMC_KEYS entry from the profiled bench lines, and
    none when the passes disagree (a library rebuilt between passes)."""
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("summ", os.path.join(ROOT, "tools", "summarize_profile.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    line = {"dtype": "f32", "build": {"lib_sha256": WANT["lib_sha256"]},
            "config": {"envs_per_gpu": 65536, "action_repeats": 3, "action_kind": "discrete",
                       "kernel_shape": {"step": "throughput", "reset": "throughput"}}}
    for sub in ("trace", "fetch", "write"):
        (tmp_path / f"{sub}.json").write_text("noise\n" + json.dumps(line) + "\n")
    w = m.workload_keys(str(tmp_path))
    assert w == WANT and set(w) == set(bench.PMC_KEYS)
    line["build"]["lib_sha256"] = "ef" * 32
    (tmp_path / "write.json").write_text(json.dumps(line) + "\n")
    assert m.workload_keys(str(tmp_path)) is None
