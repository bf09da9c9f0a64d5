"""CPU: the bench contract line and the `--gpus N` launcher (VERDICT r3 "do this" 1 and 2).

* The formatter turns a full result dict (every leg, as bench.py assembles it) into a last
  stdout line that is strict JSON and under 8 KB, with the headline's roofline and
  cpu_baseline; NaN/inf become null.
* `bench.py --gpus 2 --dry-run-cpu` without a launcher starts two gloo ranks through
  torch.distributed.run (a child process) and prints one contract line with n_gpus = 2; a
  WORLD_SIZE that disagrees with --gpus exits non-zero.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench_report  # noqa: E402


def _full_result():
    """A round-3 bench result (23 KB, every leg) from profiles/, or a synthetic one."""
    f = ROOT / "profiles" / "r03_final2_bench.json"
    if f.exists():
        return json.loads(f.read_text())
    leg = {"value": 1.0, "unit": "x/s", "roofline": {"frac": 0.1, "bound": "hbm", "basis": "b" * 500},
           "cpu_baseline": {"cores_1": {"value": 1.0}, "cores_16": {"value": 2.0}}}
    out = {"metric": "m", "value": 1.0, "unit": "u", "n_gpus": 1, "steps": 20, "warmup": 5,
           "ms_per_step": 0.04, "config": {"workload": "w", "Na": 20000, "Nz": 7},
           "roofline": {"bound": "valu", "achieved": 1, "peak": 78.6, "frac": 0.01},
           "cpu_baseline": {"value": 1.0, "cores": 16, "kind": "port", "sample": "s"}}
    for n in range(30):
        out[f"leg{n}"] = dict(leg, detail="x" * 800)
    return out


def test_contract_line_is_small_strict_json():
    out = _full_result()
    assert len(json.dumps(out)) > 8000  # the round-3 line that the driver could not parse
    line = bench_report.contract_line(out, "gpurun_out/bench_detail.json")
    assert len(line.encode()) < 8000 and "\n" not in line
    c = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype",
              "config", "roofline", "cpu_baseline"):
        assert k in c, k
    assert c["value"] == out["value"] and c["roofline"]["frac"] == out["roofline"]["frac"]
    assert c["cpu_baseline"]["value"] == out["cpu_baseline"]["value"]
    assert c["config"]["Na"] == 20000 and c["config"]["Nz"] == 7
    # one scalar summary per leg
    names = {n for n, _ in bench_report.legs_of(out)}
    assert set(c["legs"]) == names and len(names) >= 5


def test_contract_line_non_finite_and_oversize():
    out = {"metric": "m", "value": float("nan"), "unit": "u", "n_gpus": 1,
           "roofline": {"frac": float("inf")}, "config": {"workload": "w" * 100},
           "cpu_baseline": {"value": 1.0, "sample": "s" * 3000}}
    for n in range(200):  # far too many legs: the line still fits (legs shrink, then go)
        out[f"leg{n}"] = {"value": float(n), "unit": "u" * 30, "roofline": {"frac": 0.5},
                          "wall_ms": 1.0}
    line = bench_report.contract_line(out)
    assert len(line.encode()) < 8000
    c = json.loads(line)
    assert c["value"] is None and c["roofline"]["frac"] is None


def test_detail_file_strict_json(tmp_path):
    out = {"value": float("nan"), "a": [1.0, float("-inf")], "b": {"c": 2}}
    p = tmp_path / "d" / "detail.json"
    bench_report.write_detail(out, p)
    d = json.loads(p.read_text())
    assert d == {"value": None, "a": [1.0, None], "b": {"c": 2}}


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def test_gpus_two_launches_two_ranks():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dry-run-cpu",
                        "--steps", "3", "--warmup", "1"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    c = json.loads(r.stdout.strip().splitlines()[-1])
    assert c["n_gpus"] == 2 and c["steps"] == 3 and c["value"] > 0


def test_world_mismatch_exits_nonzero():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dry-run-cpu"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


@pytest.mark.parametrize("script", ["bench_ks.py", "bench_ge.py"])
def test_side_benches_refuse_world_mismatch(script):
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / script), "--gpus", "4"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_failed_leg_is_reported():
    """A leg that raised (e.g. the N > 1 `ks_direct` leg) appears in the line with its error."""
    out = {"metric": "m", "value": 1.0, "unit": "u", "n_gpus": 2, "steps": 1, "warmup": 0,
           "ms_per_step": 1.0, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f64", "data": "synthetic", "config": {"workload": "w"},
           "ks_direct": {"error": "DirectPeers: IPC mapping: " + "x" * 500}}
    line = bench_report.contract_line(out)
    d = json.loads(line)
    assert d["legs"]["ks_direct"]["error"].startswith("DirectPeers: IPC mapping")
    assert len(d["legs"]["ks_direct"]["error"]) <= 160
