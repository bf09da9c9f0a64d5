"""Where the staged KS sweep's time goes (one GPU, the direct model's shard with the most peer
columns, k = 32,768, K = 64, 8 (K, Z) shards): GPU time per sweep of
  plain   the fused sweep over the shard's nodes (ks_dev_howard_fused, no split)
  parts   interior launch + boundary launch (ks_dev_howard_fused_part 0, 1)
  one     ks_dev_staged_sweep without halo copies and without flags (both lists in one launch)
  copy    ... with the halo copies (boundary rows wait for them), no flags
  pub     ... + flags: publish only (mask 0)
  full    ... + the self-satisfied wait (mask = own slot)
Prints one JSON line (us per sweep)."""
import ctypes as C
import json
import mmap
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main(nk=32768, nK=64, world=8, sweeps=24):
    import torch
    import bench
    pkg = bench.load_pkg()
    kd = pkg.ks_dist
    dev = torch.device("cuda", 0)
    kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=nk, K_size=nK)
    B = np.array([0.1, 0.97, 0.08, 0.975])
    V = torch.as_tensor(np.ascontiguousarray(V0.transpose(2, 1, 0)), device=dev)
    slices = [kd.shard_slices(nK, q, world) for q in range(world)]
    owner = [0] * (4 * nK)
    for q, (K0, K1, s0, s1) in enumerate(slices):
        for sidx in range(s0, s1):
            for K in range(K0, K1):
                owner[sidx * nK + K] = q
    plans = []
    for q in range(world):
        K0, K1, s0, s1 = slices[q]
        own = [sidx * nK + K for sidx in range(s0, s1) for K in range(K0, K1)]
        kp = kd.forecast_index(Kg, B, pkg.ks_params())
        plans.append(kd.staged_plan(own, kp, owner, nK, q))
    q = max(range(world), key=lambda x: len(plans[x][0]))
    remote, interior, boundary = plans[q]
    sh = kd.HipShard(kg, Kg, B, P, pkg.ks_params(), *slices[q])
    ko = torch.ones_like(V)
    dV = torch.empty_like(V)
    sh.improve(V, ko)
    sh.slopes(V, dV)
    Vb = [V.clone() for _ in range(3)]
    dVb = [dV.clone() for _ in range(3)]
    nr = len(remote)
    cb = 8 * nk
    hV = torch.empty((max(nr, 1), nk), dtype=torch.float64, device=dev)
    hdV = torch.empty_like(hV)
    slot = {c: i for i, c in enumerate(remote)}
    tabs = [torch.tensor([(hV.data_ptr() + cb * slot[c]) if c in slot else Vb[b].data_ptr() + cb * c
                          for c in range(4 * nK)] +
                         [(hdV.data_ptr() + cb * slot[c]) if c in slot else dVb[b].data_ptr() + cb * c
                          for c in range(4 * nK)], dtype=torch.int64, device=dev) for b in range(3)]
    peer = V.clone()
    peerd = dV.clone()
    arr = lambda xs: torch.tensor(xs or [0], dtype=torch.int64, device=dev)
    src = arr([peer.data_ptr() + cb * c for c in remote] + [peerd.data_ptr() + cb * c for c in remote])
    dst = arr([hV.data_ptr() + cb * i for i in range(nr)] + [hdV.data_ptr() + cb * i for i in range(nr)])
    page = mmap.mmap(-1, 16384)
    host = C.c_char.from_buffer(page)
    hp = C.addressof(host)
    dptr = C.c_void_p()
    check, lib = pkg._capi.check, pkg._capi.lib
    check(lib().aiy_host_register(C.c_void_p(hp), C.c_int64(16384), C.byref(dptr)))
    C.c_uint64.from_address(hp).value = 1
    ev = lambda: torch.cuda.Event(enable_timing=True)
    st = {"v": 1}

    def run(mode, n):
        for i in range(n):
            b, bo = i % 3, (i + 1) % 3
            if mode == "plain":
                sh.set_columns(None)
                sh.howard_fused(Vb[b], dVb[b], ko, Vb[bo], dVb[bo])
                continue
            sh.set_columns(tabs[b])
            if mode == "parts":
                for part in (0, 1):
                    check(lib().ks_dev_howard_fused_part(sh._h, C.c_int(part),
                          C.c_void_p(Vb[b].data_ptr()), C.c_void_p(dVb[b].data_ptr()),
                          C.c_void_p(ko.data_ptr()), C.c_void_p(Vb[bo].data_ptr()),
                          C.c_void_p(dVb[bo].data_ptr()), pkg._capi.stream_handle(None)))
                continue
            halo = mode != "one"
            kw = {}
            if mode in ("pub", "full"):
                v = st["v"]
                kw = dict(flags=dptr.value, mask=1 if mode == "full" else 0, wait_v=v, slot=0,
                          pub_v=v, err=dptr.value + 8192)
                st["v"] = v + 1
            sh.staged_sweep(Vb[b], dVb[b], ko, Vb[bo], dVb[bo], src if halo else None,
                            dst if halo else None, 2 * nr if halo else 0, **kw)
        sh.set_columns(None)

    out = {"shard": q, "remote": nr, "interior": len(interior), "boundary": len(boundary)}
    sh.set_split(interior, boundary)
    for rep in range(2):
        for mode in ("plain", "parts", "one", "copy", "pub", "full"):
            run(mode, 3)
            torch.cuda.synchronize()
            e0, e1 = ev(), ev()
            e0.record()
            run(mode, sweeps)
            e1.record()
            torch.cuda.synchronize()
            out[f"{mode}_us"] = round(e0.elapsed_time(e1) / sweeps * 1e3, 2)
    out["timeout_word"] = C.c_uint64.from_address(hp + 8192).value
    check(lib().aiy_host_unregister(C.c_void_p(hp)))
    del host
    page.close()
    sh.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
