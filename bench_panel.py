"""F3/F2 bench: the Krusell-Smith shock panel (Krusell_Smith_VFI.m:57-94) and the agent-panel
capital simulation (:206-248) on one MI355X, inputs resident in HBM.

    python bench_panel.py [--T 1100] [--pop 10000] [--big-pop 1000000] [--big-T 200]

Two sizes: the script's own panel (T = 1100 periods, 10,000 agents, MATLAB's rand stream) and
a scaled panel (default 10^6 agents x 200 periods, device-generated uniforms — the kernels do
not depend on the values' origin).  Unit = one agent-period.  Algorithmic HBM bytes per
agent-period: shocks 9 (one fp64 uniform read, one int8 state written); simulation 17 (int8
state, fp64 capital read and written; grids and k_opt live in LDS/L2).  Prints one JSON line;
bench.py embeds the same dict as `ks_panel`."""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md
BYTES_SHOCK = 9
BYTES_SIM = 17


def _policy(kg, Kg):
    """A policy of the script's shape (k x K x 4, increasing in k, employed save more) whose
    aggregate path moves: k' = 0.95 k + 2 - 0.5 [unemployed] + 0.01 (K - 40)."""
    import numpy as np
    unemp = np.array([0.0, 1.0, 0.0, 1.0])
    return (0.95 * kg[:, None, None] + 2.0 - 0.5 * unemp[None, None, :]
            + 0.01 * (Kg[None, :, None] - 40.0))


def _time(fn, reps):
    import torch
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ms = []
    for _ in range(reps):
        torch.cuda.synchronize()
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        ms.append(ev[0].elapsed_time(ev[1]))
    ms.sort()
    return ms[len(ms) // 2]


def panel_leg(pkg, dev, T=1100, pop=10000, big_T=200, big_pop=1_000_000, reps=5, cpu_threads=None):
    """Both panel sizes on the GPU; with cpu_threads set, the restatement's CPU figure on the
    script's panel as `cpu_baseline` (numpy, one thread — it vectorises over agents, not
    cores), and `value` = the script-size panel's agent-periods/s (shocks + simulation)."""
    import numpy as np
    import torch
    kp = pkg.ks_panel
    prm = pkg.ks_params()
    kg, Kg, P, V0 = pkg.calibration.krusell_smith()
    k_opt = _policy(kg, Kg)
    ko = torch.as_tensor(np.ascontiguousarray(k_opt.transpose(2, 1, 0)), device=dev)
    kg_t, Kg_t = torch.as_tensor(kg, device=dev), torch.as_tensor(Kg, device=dev)
    out = {}
    for name, TT, nn, ustream in (("reference", T, pop, "matlab"), ("scaled", big_T, big_pop, "device")):
        n_u = kp.shock_draws(TT, nn)
        if ustream == "matlab":
            U = torch.as_tensor(kp.matlab_rand(n_u), device=dev)
        else:
            g = torch.Generator(device=dev)
            g.manual_seed(5489)
            U = torch.rand(n_u, dtype=torch.float64, device=dev, generator=g)
        zi, eps = kp.ks_shocks_dev(U, prm, TT, nn)   # warm-up
        t_sh = _time(lambda: kp.ks_shocks_dev(U, prm, TT, nn), reps)
        k0 = torch.full((nn,), float(Kg[0]), dtype=torch.float64, device=dev)
        sim = kp.PanelSim(kg_t, Kg_t, zi, eps, k0.clone())
        sim(ko)
        torch.cuda.synchronize()

        def run():
            sim.k_pop.copy_(k0)
            sim(ko)
        t_sim = _time(run, reps)
        units = TT * nn
        bw_sh = BYTES_SHOCK * units / (t_sh * 1e-3) / 1e9
        bw_sim = BYTES_SIM * units / (t_sim * 1e-3) / 1e9
        out[name] = {
            "T": TT, "population": nn, "uniforms": ustream,
            "shocks_ms": t_sh, "shocks_agent_periods_per_s": units / (t_sh * 1e-3),
            "shocks_roofline": {"bound": "hbm", "achieved": bw_sh, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": bw_sh / HBM_PEAK_GBS,
                                "basis": f"{BYTES_SHOCK} B per agent-period"},
            "simulate_ms": t_sim, "simulate_agent_periods_per_s": units / (t_sim * 1e-3),
            "simulate_us_per_period": t_sim * 1e3 / max(TT - 1, 1),
            "simulate_roofline": {"bound": "hbm", "achieved": bw_sim, "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": bw_sim / HBM_PEAK_GBS,
                                  "basis": f"{BYTES_SIM} B per agent-period; {TT - 1} "
                                           f"dependent periods (one launch each)"},
            "K_ts_last": float(sim.K_ts[-1]),
        }
        del U, zi, eps, sim
        torch.cuda.empty_cache()
    ref = out["reference"]
    res = {"metric": "Krusell-Smith panel agent-periods/s (shocks + capital simulation, fp64)",
           "workload": "Krusell_Smith_VFI.m:57-94 and :206-248", **out,
           "value": ref["T"] * ref["population"] / ((ref["shocks_ms"] + ref["simulate_ms"]) * 1e-3),
           "unit": "agent-periods/s (script panel, shocks + simulation)"}
    if cpu_threads is not None:
        c = cpu_leg(T, pop)
        res["cpu_baseline"] = {"value": c["agent_periods_per_s"], "unit": "agent-periods/s",
                               "cores": 1, "kind": "port", **c,
                               "sample": f"the script's panel (T={T}, {pop} agents): numpy "
                                         f"restatement (oracle/np_oracle.py ks_shocks + "
                                         f"ks_panel_simulate), one thread"}
    return res


def cpu_leg(T=1100, pop=10000):
    """The numpy restatement (oracle, 1 thread, vectorised over agents) on the script's panel."""
    import time
    import numpy as np
    from oracle import np_oracle as no
    p, kg, Kg, *_ = no.ks_setup()
    k_opt = _policy(kg, Kg)
    U = no.matlab_rand_stream(no.ks_shock_draws(T, pop))
    t0 = time.perf_counter()
    zi, e = no.ks_shocks(p, T, pop, U)
    t1 = time.perf_counter()
    no.ks_panel_simulate(kg, Kg, k_opt, zi, e, np.full(pop, Kg[0]))
    t2 = time.perf_counter()
    return {"kind": "port (numpy restatement, vectorised over agents)", "cores": 1,
            "shocks_s": t1 - t0, "simulate_s": t2 - t1,
            "agent_periods_per_s": T * pop / (t2 - t0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=1100)
    ap.add_argument("--pop", type=int, default=10000)
    ap.add_argument("--big-T", type=int, default=200)
    ap.add_argument("--big-pop", type=int, default=1_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = panel_leg(bench.load_pkg(), dev, args.T, args.pop, args.big_T, args.big_pop)
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_leg(args.T, args.pop)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
