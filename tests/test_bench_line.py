"""bench.py's stdout contract: ONE JSON line the driver can parse (round 3's
22.9 KB line was not parsed), with the headline fields,
its roofline and cpu_baseline; the per-level traces and notes go to the
detail file.  Built here from the committed round-3 full record (a canned
stats object of the old, verbose format)."""
import json
import sys
from types import SimpleNamespace

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (stdlib-only at import time)

CANNED = ROOT / "profiles" / "r03" / "bench_default.json"


def _canned():
    d = json.loads(CANNED.read_text())
    head = {k: d[k] for k in ("value", "ms_per_frame", "rays_per_frame", "roofline", "trace", "ms_1spp", "bvh",
                              "scene_build_ms")}
    head["scene"] = d["config"]["scene"]
    head["batch_paths"] = d["config"]["batch_paths"]
    head["roofline_other"] = []
    # (round 5: traced rays only in value, host-culled camera rays beside it;
    # the round-3 record predates the field)
    head["culled_rays_per_frame"] = 0
    for o in d["configs"]:
        o.setdefault("culled_rays_per_frame", 0)
    return head, d["configs"], d["cpu_baseline"]


ARGS = SimpleNamespace(width=1024, height=1024, spp=256, bounces=8, steps=3, warmup=1, seed=15618,
                       scene="CBempty", tile=32)


def test_line_is_bounded_and_complete():
    head, others, cpu = _canned()
    # the verbose record is what broke the driver
    assert len(json.dumps(bench.detail_record(head, others, cpu, ARGS, 1))) > bench.LINE_MAX
    line = bench.compact_line(head, others, cpu, ARGS, 1, detail_path="gpurun_out/bench_detail.json")
    assert "\n" not in line and len(line) < 12000
    out = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "culled_rays_per_frame"):
        assert k in out, k
    assert out["value"] == head["value"] and out["ms_per_step"] == head["ms_per_frame"]
    r = out["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    c = out["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert len(out["configs"]) == len(others)
    for o, c in zip(others, out["configs"]):
        assert c["scene"] == o["scene"] and c["value"] == o["value"]
        assert c["culled_rays_per_frame"] == o["culled_rays_per_frame"]
        assert set(c["roofline"]) == {"kernel", "frac", "achieved", "traffic"}
    assert out["detail"] == "gpurun_out/bench_detail.json"


def test_line_bounded_with_many_workloads():
    """Even a line with 4x the workloads stays under the bound (the extras
    are dropped before the headline fields)."""
    head, others, cpu = _canned()
    line = bench.compact_line(head, others * 4, cpu, ARGS, 1)
    assert len(line) < 12000
    out = json.loads(line)
    assert out["roofline"]["frac"] > 0 and "cpu_baseline" in out


def test_visible_gpus_from_sysfs(tmp_path):
    """The rank launcher counts GPUs from the KFD topology (no HIP runtime in
    the parent process), narrowed by the visibility variables."""
    for i, simds in enumerate([0, 1024, 1024, 0, 1024]):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 8\nsimd_count {simds}\nmem_banks_count 1\n")
    assert bench.visible_gpus(tmp_path, env={}) == 3
    assert bench.visible_gpus(tmp_path, env={"HIP_VISIBLE_DEVICES": "0,1"}) == 2
    assert bench.visible_gpus(tmp_path, env={"ROCR_VISIBLE_DEVICES": ""}) == 0
    assert bench.visible_gpus(tmp_path / "missing", env={}) == 0


def test_line_carries_executed_work():
    """The k_path_leaf roofline reports the work the kernel executes (the
    PT_FLAG_COUNT_TESTS frame: executed_flop per launch, executed_frac) beside
    the reference's per-ray work (achieved / frac), VERDICT r5 item 3."""
    head, others, cpu = _canned()
    r = dict(head["roofline"])
    r.update({"kernel": "k_path_leaf", "executed_flop": 123456789, "executed_achieved": 30.0,
              "executed_frac": round(30.0 / bench.VALU_PEAK_TFLOPS, 4), "executed_tests_per_ray": 2.5})
    head["roofline"] = r
    out = json.loads(bench.compact_line(head, others, cpu, ARGS, 1))
    ro = out["roofline"]
    for k in ("executed_flop", "executed_frac", "executed_tests_per_ray", "frac", "achieved"):
        assert k in ro, k
    assert abs(ro["executed_frac"] - 30.0 / bench.VALU_PEAK_TFLOPS) < 1e-4
    assert bench.FLOP_TRI == 42 and bench.FLOP_SPHERE == 19 and bench.FLOP_BOX == 12
