"""The bench contract line and the detail file (VERDICT r3 "do this" 1).

bench.py assembles one large result dict (the headline plus every leg: labour VFI, EGM, the
config-4 batch, A10 pushes, KS sharded, KS panel, GE walls, CPU baselines).  The driver keeps
only the tail of stdout, so the full dict goes to a detail file and the LAST stdout line is a
compact, strict-JSON contract line (< 8 KB) holding the contract fields, the headline roofline
and cpu_baseline, and one scalar summary per leg.

    contract(out, detail_path) -> dict      the compact line's object
    contract_line(out, detail_path) -> str  json.dumps(..., allow_nan=False), < MAX_BYTES
    write_detail(out, path)                 the full dict (non-finite numbers -> null)
"""
from __future__ import annotations

import json
import math
import os

MAX_BYTES = 8000

# contract fields copied verbatim when present
TOP = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
       "scaling", "vs_baseline", "dtype", "data")
CONFIG = ("workload", "Na", "Nz", "parallelism", "search", "sweeps_timed")
ROOF = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_avg_ms",
        "effective_frac_d3", "pmc_source")
CPU = ("value", "unit", "cores", "kind", "sample")


def finite(x):
    """A copy of x with NaN/inf replaced by None (strict JSON)."""
    if isinstance(x, float):
        return x if math.isfinite(x) else None
    if isinstance(x, dict):
        return {str(k): finite(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [finite(v) for v in x]
    if hasattr(x, "item") and not isinstance(x, (str, bytes)):  # numpy scalars
        try:
            return finite(x.item())
        except (TypeError, ValueError):
            return str(x)
    return x


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def _num(x):
    return x if isinstance(x, (int, float)) and not isinstance(x, bool) else None


def _cpu_value(cb):
    """The all-cores CPU figure of a leg's cpu_baseline (value, or the largest cores_N)."""
    if not isinstance(cb, dict):
        return None, None
    if _num(cb.get("value")) is not None:
        return cb["value"], cb.get("cores")
    best = None
    for k, v in cb.items():
        if k.startswith("cores_") and isinstance(v, dict) and _num(v.get("value")) is not None:
            n = int(k[6:]) if k[6:].isdigit() else 0
            if best is None or n > best[1]:
                best = (v["value"], n)
    return best if best else (None, None)


def leg_summary(leg):
    """One line of scalars for a leg: value/unit, roofline frac (+ bound), the CPU figure."""
    s = {}
    if _num(leg.get("value")) is not None:
        s["value"] = leg["value"]
        if "unit" in leg:
            s["unit"] = leg["unit"]
    rf = leg.get("roofline")
    if isinstance(rf, dict) and _num(rf.get("frac")) is not None:
        s["frac"] = rf["frac"]
        s["bound"] = rf.get("bound")
    # the counter pass behind the leg's PMC block: its first file's name (profiles/<round>_pmc_*)
    src = (rf or {}).get("pmc_source") if isinstance(rf, dict) else None
    src = src or leg.get("pmc_source")
    if isinstance(src, str) and src:
        s["pmc"] = src.split(",")[0].split(" ")[0].replace("profiles/", "")
    cv, cores = _cpu_value(leg.get("cpu_baseline"))
    if cv is not None:
        s["cpu"] = cv
        s["cpu_cores"] = cores
    if isinstance(leg.get("error"), str):   # a leg that failed says so in the line
        s["error"] = leg["error"][:160]
    for k in ("wall_s_gpu", "wall_s_cpu", "identical_trace", "r", "r_gpu", "iters", "wall_ms",
              "ms_per_sweep", "us_per_step", "us_per_push", "howard_ms_per_sweep",
              "vfi_iteration_ms", "r_equals_reference_trace", "speedup_vs_sequential_rates",
              "bit_exact_vs_halo", "hw_queues", "wall_s_gpu_inherited_queues"):
        if k in leg and (_num(leg[k]) is not None or isinstance(leg[k], bool)):
            s[k] = leg[k]
    return s


def legs_of(out):
    """Every leg of the result dict as (name, dict): top-level dicts that carry a value or a
    roofline, and one level below for size-keyed legs (egm.Na20000, labor_vfi.Na400, ...)."""
    skip = {"config", "roofline", "repeats", "cpu_baseline"}
    for name, v in out.items():
        if name in skip or not isinstance(v, dict):
            continue
        if "value" in v or "roofline" in v or "wall_s_gpu" in v or "iters" in v or "error" in v:
            yield name, v
        else:
            for sub, w in v.items():
                if isinstance(w, dict) and ("value" in w or "roofline" in w):
                    yield f"{name}.{sub}", w


def contract(out, detail_path=None):
    c = _pick(out, TOP)
    c["config"] = _pick(out.get("config", {}), CONFIG)
    rf = _pick(out.get("roofline", {}), ROOF)
    if rf:
        c["roofline"] = rf
    cb = out.get("cpu_baseline")
    if isinstance(cb, dict):
        c["cpu_baseline"] = _pick(cb, CPU)
        oc = cb.get("one_core")
        if isinstance(oc, dict):
            c["cpu_baseline"]["one_core"] = oc.get("value")
    rep = out.get("repeats")
    if isinstance(rep, dict):
        c["repeats"] = _pick(rep, ("n", "min_ms_per_step", "max_ms_per_step"))
    legs = {n: leg_summary(v) for n, v in legs_of(out)}
    if legs:
        c["legs"] = legs
    if detail_path:
        c["detail"] = str(detail_path)
    return finite(c)


def contract_line(out, detail_path=None, max_bytes=MAX_BYTES):
    """The compact line; shrinks (leg extras, then samples, then legs) until < max_bytes."""
    c = contract(out, detail_path)
    line = json.dumps(c, allow_nan=False, separators=(",", ":"))
    if len(line.encode()) < max_bytes:
        return line
    for v in c.get("legs", {}).values():  # keep value/unit/frac/cpu only
        for k in list(v):
            if k not in ("value", "unit", "frac", "cpu"):
                del v[k]
    line = json.dumps(c, allow_nan=False, separators=(",", ":"))
    if len(line.encode()) < max_bytes:
        return line
    if "cpu_baseline" in c:
        c["cpu_baseline"].pop("sample", None)
    c["config"] = {k: c["config"][k] for k in ("workload", "Na", "Nz") if k in c["config"]}
    c.get("roofline", {}).pop("pmc_source", None)
    line = json.dumps(c, allow_nan=False, separators=(",", ":"))
    if len(line.encode()) < max_bytes:
        return line
    c.pop("legs", None)
    return json.dumps(c, allow_nan=False, separators=(",", ":"))


def write_detail(out, path):
    path = os.fspath(path)
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "w") as f:
        json.dump(finite(out), f, allow_nan=False, indent=1)
