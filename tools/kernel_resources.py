"""Per-kernel register / scratch / occupancy report of the gfx950 build (compiler remarks):

    python tools/kernel_resources.py [file.hip ...]     (default: every csrc/*_kernels.hip)

Prints one line per kernel: VGPRs, AGPRs, scratch bytes per lane, spills, LDS, occupancy.  A
kernel with scratch > 0 pays vector-memory round trips for private arrays or spills."""
import glob
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "aiyagari-replication_amd" / "csrc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fno-fast-math", "-Rpass-analysis=kernel-resource-usage", "-c", "-o", "/dev/null"]


def report(src):
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, str(Path(src).resolve())], capture_output=True, text=True,
                       cwd=CSRC)
    cur, rows = None, []
    for ln in r.stderr.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", ln)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s*(\S+) \[-Rpass", ln)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    return rows


def main():
    srcs = sys.argv[1:] or sorted(glob.glob(str(CSRC / "*_kernels.hip")))
    for s in srcs:
        for k in report(s):
            dem = subprocess.run(["c++filt", k["name"]], capture_output=True, text=True).stdout.strip()
            print(f"{Path(s).name:22s} vgpr {k.get('VGPRs', '?'):>4} agpr {k.get('AGPRs', '?'):>3} "
                  f"scratch {k.get('ScratchSize [bytes/lane]', '?'):>4} "
                  f"sgpr-spill {k.get('SGPRs Spill', '?'):>3} vgpr-spill {k.get('VGPRs Spill', '?'):>3} "
                  f"lds {k.get('LDS Size [bytes/block]', '?'):>6} occ {k.get('Occupancy [waves/SIMD]', '?'):>2}  "
                  f"{dem[:110]}")


if __name__ == "__main__":
    main()
