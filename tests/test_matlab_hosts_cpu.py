"""B6: the committed MATLAB/Octave host scripts (aiyagari-replication_amd/matlab/*.m) call the
gateways with argument and output counts each gateway accepts, and are structurally well formed
(balanced blocks and brackets).  Neither MATLAB nor Octave exists in this image, so this is the
"stub flow" check: the calls are matched against the gateways' own aiy_nargs bounds, parsed from
their C sources — the same bounds the stub-linked gateways enforce in tests/test_mex_*.py."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
MEX = ROOT / "aiyagari-replication_amd" / "mex"
SCRIPTS = sorted((ROOT / "aiyagari-replication_amd" / "matlab").glob("*.m"))


def gateway_bounds():
    out = {}
    for f in MEX.glob("*_mex.c"):
        m = re.search(r"aiy_nargs\(nrhs, (\d+), (\d+), nlhs, (\d+),", f.read_text())
        out[f.stem] = (int(m.group(1)), int(m.group(2)), int(m.group(3)))
    return out


def _strip(src):
    """Drop comments and string literals (MATLAB: % to end of line; '...' strings)."""
    lines = []
    for ln in src.splitlines():
        ln = re.sub(r"'[^'\n]*'", "''", ln)
        ln = ln.split("%", 1)[0]
        lines.append(ln)
    return "\n".join(lines)


def _join_continuations(src):
    return re.sub(r"\.\.\.\s*\n", " ", src)


def _split_args(s):
    depth, cur, parts = 0, "", []
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur)
    return parts


def _calls(src):
    """(gateway, nargin, nargout) for every `[a, b] = name_mex(...)` / `x = name_mex(...)`."""
    out = []
    for m in re.finditer(r"(?:\[([^\]]*)\]|(\w+))\s*=\s*(\w+_mex)\s*\(", src):
        lhs = m.group(1) if m.group(1) is not None else m.group(2)
        nout = len([x for x in lhs.split(",") if x.strip()])
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        out.append((m.group(3), len(_split_args(src[m.end():i - 1])), nout))
    return out


@pytest.mark.parametrize("script", SCRIPTS, ids=lambda p: p.name)
def test_gateway_calls_match_gateway_signatures(script):
    bounds = gateway_bounds()
    src = _join_continuations(_strip(script.read_text()))
    calls = _calls(src)
    assert calls, "the host script calls no gateway"
    for name, nin, nout in calls:
        assert name in bounds, f"{name}: no such gateway in mex/"
        lo, hi, maxl = bounds[name]
        assert lo <= nin <= hi, f"{name}: {nin} inputs, gateway takes {lo}..{hi}"
        assert nout <= maxl, f"{name}: {nout} outputs, gateway gives {maxl}"


@pytest.mark.parametrize("script", SCRIPTS, ids=lambda p: p.name)
def test_script_blocks_and_brackets_balance(script):
    src = _join_continuations(_strip(script.read_text()))
    for a, b in ("()", "[]", "{}"):
        assert src.count(a) == src.count(b), (a, b)
    opens = len(re.findall(r"^\s*(for|while|if|switch|function|try)\b", src, flags=re.M))
    ends = len(re.findall(r"^\s*end\s*;?\s*$", src, flags=re.M))
    assert opens == ends, (opens, ends)


def test_every_script_is_covered():
    names = {p.name for p in SCRIPTS}
    assert {"aiyagari_vfi_gpu.m", "aiyagari_ge_multisection_gpu.m", "aiyagari_labor_vfi_gpu.m",
            "aiyagari_egm_gpu.m", "aiyagari_labor_egm_gpu.m", "krusell_smith_vfi_gpu.m",
            "krusell_smith_egm_gpu.m"} <= names


def test_every_gateway_is_called_by_a_host_script():
    """Every gateway in mex/ (the replacement for one inner loop of one reference script) is
    called by at least one committed host script."""
    called = set()
    for f in SCRIPTS:
        called |= {c[0] for c in _calls(_join_continuations(_strip(f.read_text())))}
    assert set(gateway_bounds()) - called == set()
