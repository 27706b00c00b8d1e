"""The reference glue optimiser's own sensitivity envelope: how far its
result moves under input perturbations far below anything physical, so that the device
optimiser's tolerance is stated in the reference's own terms instead of the device's tails.

The reference optimiser is oracle/glue.py (a torch restatement that reproduces the
reference's LBFGS optimum bit for bit on the fixtures: tests/test_glue.py::
test_oracle_matches_reference_optimum).  Each variant runs the fixture's whole reference
sequence on the host -- RmsdBPE with the oracle's numpy NeRF / Kabsch and this optimiser in
place of the device batches, exactly tests/test_glue.py's host path -- with ONE change to the
optimiser's inputs:

  ref        none (must reproduce the fixture exactly: the control)
  x0_up/dn   every start value x0 moved 1 float32 ulp up / down
  tgt_up     every target frame value (R, t; float32 in the optimiser) 1 ulp up
  geo_up     every fixed geometry value of the chain (float32 in the optimiser) 1 ulp up
  threads    torch.set_num_threads(8) instead of 1 (summation order of torch's kernels)
  grad_s<k>  at EVERY evaluation the gradient the closure returns moved 1 float32 ulp up or
             down per element (random signs, seed k): another float32 gradient of the same
             loss, as a different summation order or rounding point gives one
  eval_s<k>  as grad_s<k>, and the loss value the closure returns moved 1 ulp too (random
             sign): another float32 evaluation of loss AND gradient -- the model of an
             independent float32 implementation of the optimiser (such as the device's),
             whose loss feeds the strong-Wolfe line search's comparisons

Recorded per (fixture, variant): after glue_opt_all, the glued geometry against the
fixture's (the reference's): glues in another bin, their distance (rad), how many further
than 0.02 / 0.1 rad, per glue type; then the merges popped by bin() + step() and how many
leading merges equal the fixture's.  And for the 120-chain drift set (tools/glue_drift.py,
prior off) the raw optimum's drift quantiles and same-bin share against the unperturbed
optimum.

  python tools/glue_envelope.py [--jobs N] [--no-steps] [--variants a,b] OUT.json [fixture ...]
  python tools/glue_envelope.py --merge OUT.json LOG ...   (the result lines of earlier runs)

CPU only, run in the build container (torch on the CPU); the output is committed as
tests/golden/glue_envelope.json and tests/test_glue.py derives its device bounds from it.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "pt-bpe_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

FIXTURES = ["gl_all_p0", "gl_all_p0_prior", "gl_pdb72_readme", "gl_syn120_pareto"]
VARIANTS = ["ref", "x0_up", "x0_dn", "tgt_up", "geo_up", "threads", "grad_s0", "grad_s1", "grad_s2",
            "eval_s0", "eval_s1", "eval_s2"]
GLUE_COLS = ["omega", "C:1N:1CA", "phi"]
COLS = ["0C:1N", "N:CA", "CA:C", "phi", "psi", "omega", "tau", "CA:C:1N", "C:1N:1CA"]


def _up(a):
    a = np.asarray(a, dtype=np.float32)
    return np.nextafter(a, np.float32(np.inf)).astype(np.float32)


def _dn(a):
    a = np.asarray(a, dtype=np.float32)
    return np.nextafter(a, np.float32(-np.inf)).astype(np.float32)


def optimize_grad_ulp(geo, x0, R_occs, t_occs, prior, lam, rng, loss_too=False):
    """oracle.glue.optimize with every gradient the closure hands LBFGS moved 1 float32 ulp
    (random direction per element); loss_too: the loss value it returns as well."""
    import torch
    from oracle import glue as og
    geo32 = torch.tensor(np.asarray(geo, dtype=np.float32))
    R = [torch.tensor(np.asarray(x, dtype=np.float32)) for x in R_occs]
    T = [torch.tensor(np.asarray(x, dtype=np.float32)) for x in t_occs]
    pr = None
    if prior is not None:
        pr = [(torch.tensor(np.asarray(c, dtype=np.float32)), torch.tensor(np.asarray(w, dtype=np.float32)))
              for c, w in prior]
    raw = torch.nn.Parameter(torch.tensor(np.ascontiguousarray(x0, dtype=np.float32)))
    opt = torch.optim.LBFGS([raw], max_iter=20, line_search_fn="strong_wolfe")
    losses = []

    def closure():
        opt.zero_grad()
        loss = og.chain_loss(geo32, raw, R, T, pr, lam)
        loss.backward()
        g = raw.grad.numpy()
        up = rng.random(g.shape) < 0.5
        g2 = np.where(up, np.nextafter(g, np.float32(np.inf)), np.nextafter(g, np.float32(-np.inf))).astype(np.float32)
        raw.grad.copy_(torch.from_numpy(g2))
        losses.append(loss.item())
        if loss_too:
            lv = np.float32(loss.item())
            lv = np.nextafter(lv, np.float32(np.inf if rng.random() < 0.5 else -np.inf)).astype(np.float32)
            return torch.tensor(lv)
        return loss

    opt.step(closure)
    st = opt.state[raw]
    return og.wrap(raw.detach()).numpy(), int(st["n_iter"]), int(st["func_evals"]), losses[0], losses[-1]


def perturbed_optimize(variant):
    """oracle.glue.optimize with the variant's input change."""
    from oracle import glue as og
    rng = np.random.default_rng(int(variant[6:]) if variant[:6] in ("grad_s", "eval_s") else 0)

    def opt(g, x0, R, t, prior=None, lam=0.0):
        if variant[:6] in ("grad_s", "eval_s"):
            return optimize_grad_ulp(g, x0, R, t, prior, lam, rng, loss_too=variant.startswith("eval_s"))
        if variant == "x0_up":
            x0 = _up(x0)
        elif variant == "x0_dn":
            x0 = _dn(x0)
        elif variant == "tgt_up":
            R, t = _up(R), _up(t)
        elif variant == "geo_up":
            g = _up(np.asarray(g, dtype=np.float32)).astype(np.float64)
        return og.optimize(g, x0, R, t, prior, lam)
    return opt


def install_host(variant):
    """tests/test_glue.py's host_glue fixture without pytest: the oracle's NeRF / Kabsch /
    thresholds and the (perturbed) optimiser in place of the device batches."""
    import oracle.prologue as prologue
    import oracle.rmsd as orm
    from geobpe import glue, rmsd, rmsd_bpe
    rmsd.geo_coords = lambda geos, device=0: [orm.nerf(g) for g in geos]
    rmsd.nerf_packed = lambda off, packed, device=0: orm.nerf_packed(off, packed)
    rmsd.nerf_atoms = lambda off, packed, device=0: orm.nerf_atoms(off, packed)
    rmsd.rmsd_matrix = lambda S, device=0: orm.rmsd_matrix(S)
    rmsd.rmsd_cross = lambda A, B, device=0: np.array([[orm.rmsd(a, b) for b in B] for a in A])
    rmsd_bpe.RmsdBPE._grid_thresholds = lambda self: {s: prologue.thresholds(self._corpus, b) for s, b in self.bins.items()}
    opt1 = perturbed_optimize(variant)

    def opt_chains(geos, x0s, targets, grids, prior, lam, device=0, w_rot=1.0, w_trans=0.1):
        table, counts = prior
        outs = []
        for g, x0, (R, t), gi in zip(geos, x0s, targets, grids):
            pr = [(table[gi, k, 0, :counts[gi, k]], table[gi, k, 1, :counts[gi, k]]) for k in range(3)]
            outs.append(opt1(g, x0, R, t, pr, lam)[0])
        FIRST_OPT.append(outs)
        return outs, None, None
    glue.optimize_chains = opt_chains


FIRST_OPT = []  # the raw optima of every optimize_chains call (glue_opt_all first)


def glued_stats(a, b, thr):
    """a (this run) vs b (the fixture) for one glue column: tests/test_glue.py::_glue_close's
    numbers without its asserts."""
    bad = ~((a == b) | (np.isnan(a) & np.isnan(b)))
    n = int(np.sum(~np.isnan(b)))
    e = np.asarray(thr, dtype=np.float64)
    width = float(np.max(e[:, 1] - e[:, 0]))
    d = np.abs(a[bad] - b[bad])
    d = np.minimum(d, 2 * np.pi - d)
    return {"glues": n, "other_bin": int(bad.sum()), "bin_width": width,
            "max_rad": float(d.max()) if d.size else 0.0,
            "past_0.02": int(np.sum(d > 0.02)), "past_0.1": int(np.sum(d > 0.1))}


def run_fixture(name, variant, steps=True):
    import torch
    torch.set_num_threads(8 if variant == "threads" else 1)
    install_host(variant)
    FIRST_OPT.clear()  # (a pool worker runs several jobs)
    from test_glue import _load
    from geobpe.bpe import BPE
    meta, arrs = _load(name)
    corpus = {k: arrs[k] for k in COLS + ["row_off"]}
    t0 = time.time()
    bpe = BPE(corpus, bins={int(k): v for k, v in meta["bins"].items()},
              rmsd_partition_min_size=meta["rmsd_partition_min_size"], rmsd_super_res=meta["rmsd_super_res"],
              num_partitions={int(k): v for k, v in meta["num_partitions"].items()},
              max_num_strucs=meta["max_num_strucs"], res_init=True, std_bonds=meta["std_bonds"],
              glue_opt=True, glue_opt_prior=meta["glue_opt_prior"], glue_opt_every=meta["glue_opt_every"],
              glue_opt_method=meta["glue_opt_method"], seed=meta["rng_seed"])
    popped = []
    inner = bpe._merge

    def recording():
        popped.append(list(bpe._priority[0]))
        return inner()
    bpe._merge = recording
    bpe.initialize()
    bpe.glue_opt_all()
    g = bpe.geometry()
    out = {"fixture": name, "variant": variant,
           "glued": {c: glued_stats(g[c], arrs[f"glued_{c}"], bpe._thresholds[1][c]) for c in GLUE_COLS}}
    if "lbfgs_opt" in arrs and FIRST_OPT:  # the raw optimum of glue_opt_all against the reference's
        d = np.abs(np.concatenate(FIRST_OPT[0]).astype(np.float64) - arrs["lbfgs_opt"])
        d = np.minimum(d, 2 * np.pi - d)
        out["raw_drift_rad"] = {"p50": float(np.median(d)), "p99": float(np.quantile(d, 0.99)), "max": float(d.max())}
    if steps:
        want = [p for call in meta["calls"] for p in call["popped"]]
        bpe.bin()
        for _ in meta["calls"]:
            bpe.step()
        same = next((i for i, (a, b) in enumerate(zip(popped, want)) if a != b), min(len(popped), len(want)))
        out["merges"] = {"total": len(want), "shared_prefix": same}
    out["seconds"] = round(time.time() - t0, 1)
    return out


def drift_variant(variant, n=120):
    """The drift set of tools/glue_drift.py: the variant's raw optimum against the unperturbed
    one (both the reference optimiser)."""
    import torch
    torch.set_num_threads(8 if variant == "threads" else 1)
    import glue_drift
    from geobpe import glue
    geos, x0s, R, T, thr = glue_drift.problems(n)
    z = np.load(os.path.join(REPO, "tests", "golden", "glue_drift_oracle.npz"))
    opt = perturbed_optimize(variant)
    outs, loss = [], []
    for g, x0, r, t in zip(geos, x0s, R, T):
        o = opt(g, x0, r, t)
        outs.append(o[0])
        loss.append(o[4])
    dev = np.concatenate(outs).astype(np.float64)
    ref = z["opt"].astype(np.float64)
    d = np.abs(dev - ref)
    d = np.minimum(d, 2 * np.pi - d).ravel()
    same = np.array([[glue.snap_bin(thr[t], a[t]) == glue.snap_bin(thr[t], b[t]) for t in range(3)]
                     for a, b in zip(dev, ref)])
    lr = np.array(loss) / z["loss"]
    return {"fixture": "drift120", "variant": variant, "glues": int(len(dev)),
            "drift_rad": {q: float(np.quantile(d, p)) for q, p in (("p50", .5), ("p90", .9), ("p99", .99), ("max", 1.0))},
            "exact": float(np.mean(d == 0)), "same_bin": float(same.mean()),
            "loss_ratio": {"min": float(lr.min()), "max": float(lr.max())}}


def _job(args):
    kind, name, variant, steps = args
    try:
        if kind == "drift":
            return drift_variant(variant)
        return run_fixture(name, variant, steps)
    except Exception as e:  # the reference's own failures are data too
        return {"fixture": name, "variant": variant, "raised": f"{type(e).__name__}: {e}"}


def merge_logs(out_path, logs):
    """the result lines of earlier runs' logs (one JSON object a line) into OUT.json"""
    res = {}
    if os.path.exists(out_path):
        with open(out_path) as f:
            res = {(r["fixture"], r["variant"]): r for r in json.load(f)["results"]}
    for p in logs:
        with open(p) as f:
            for ln in f:
                if ln.startswith("{"):
                    r = json.loads(ln)
                    if "fixture" in r and "variant" in r and "raised" not in r:
                        res[(r["fixture"], r["variant"])] = r
    out = sorted(res.values(), key=lambda r: (r["fixture"], VARIANTS.index(r["variant"]) if r["variant"] in VARIANTS else 99))
    with open(out_path, "w") as f:
        json.dump({"generator": "tools/glue_envelope.py", "variants": VARIANTS, "results": out}, f, indent=1)


def main(argv):
    import multiprocessing as mp
    if argv and argv[0] == "--merge":  # --merge OUT.json LOG ...
        return merge_logs(argv[1], argv[2:])
    jobs, steps, variants = 6, True, VARIANTS
    while argv and argv[0].startswith("--"):
        if argv[0] == "--jobs":
            jobs = int(argv[1])
            argv = argv[2:]
        elif argv[0] == "--no-steps":
            steps = False
            argv = argv[1:]
        elif argv[0] == "--variants":
            variants = argv[1].split(",")
            argv = argv[2:]
        else:
            raise SystemExit(f"unknown option {argv[0]}")
    out_path, names = argv[0], (argv[1:] or FIXTURES + ["drift120"])
    work = []
    for name in names:
        for v in variants:
            work.append(("drift", name, v, steps) if name == "drift120" else ("fixture", name, v, steps))
    # the longest first (the pareto fixture's runs)
    work.sort(key=lambda w: 0 if "pareto" in w[1] else (1 if "readme" in w[1] else 2))
    res = []
    with mp.get_context("spawn").Pool(jobs) as pool:
        for r in pool.imap_unordered(_job, work):
            res.append(r)
            print(json.dumps(r), flush=True)
    if os.path.exists(out_path):  # (merged with an earlier run's other variants)
        with open(out_path) as f:
            old = json.load(f)["results"]
        have = {(r["fixture"], r["variant"]) for r in res}
        res += [r for r in old if (r["fixture"], r["variant"]) not in have]
    res.sort(key=lambda r: (r["fixture"], VARIANTS.index(r["variant"]) if r["variant"] in VARIANTS else 99))
    with open(out_path, "w") as f:
        json.dump({"generator": "tools/glue_envelope.py", "variants": VARIANTS, "results": res}, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
