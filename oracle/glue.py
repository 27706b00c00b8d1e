"""CPU restatement of the reference's glue optimisation (TEST INFRASTRUCTURE: imported only
by tests/ as the checker of csrc/glue.h, never by the product path).

foldingdiff/bpe.py, restated with torch on the CPU (the reference's own numerics: float32
parameters, float32 trig, float64 atoms):
  fk_segment_torch, ret_all branch       :423-459  chain_loss (NeRF from the float32 geometry,
                                                    frames of residues 1..r-1)
  optimize_glues_entry_torch: wrap,       :462-578  optimize (torch.optim.LBFGS(max_iter=20,
    circ_kde_prior, closure, snap_bin               line_search_fn="strong_wolfe")), snap_bin
  _opt_glue_worker / opt_glue             :739-807  glue k = (omega_k, C:1N:1CA_k, phi_{k+1})
                                                    against exit frame k of the cached chain
nerf.py:151-210 (place_dihedral, torch branch) and angles_and_coords.py:586-620
(frame_from_triad_torch) are restated inline.  Pinned by tests/golden/gl_*.npz
(tests/golden/make_glue_golden.py ran the reference's optimiser and recorded its optimum).
"""
from __future__ import annotations

import bisect

import numpy as np

from .rmsd import start as _start


def _place(a, b, c, angle, length, torsion):
    import torch
    unit = lambda x: x / torch.linalg.norm(x, dim=-1, keepdim=True)  # noqa: E731
    ab = b - a
    bc = unit(c - b)
    n = unit(torch.linalg.cross(ab, bc, dim=-1))
    nbc = torch.linalg.cross(n, bc, dim=-1)
    m = torch.stack([bc, nbc, n], dim=-1)
    d = torch.stack([-length * torch.cos(angle), length * torch.cos(torsion) * torch.sin(angle),
                     length * torch.sin(torsion) * torch.sin(angle)], dim=0).type(m.dtype)
    return torch.matmul(m, d).squeeze() + c


def _normalize(v, eps=1e-8):
    return v / (v.norm(dim=-1, keepdim=True) + eps)


def _frame(N, CA, C):
    import torch
    x = _normalize(C - CA)
    u = _normalize(N - CA)
    z = _normalize(torch.cross(x, u, dim=-1))
    y = torch.cross(z, x, dim=-1)
    return torch.stack((x, y, z), dim=-1), CA.clone()


def wrap(a):
    import torch
    return torch.remainder(torch.atan2(torch.sin(a), torch.cos(a)) + (2.0 * np.pi), 2.0 * np.pi)


def circ_kde_prior(angle, centers, weights, kappa):
    import torch
    return -torch.logsumexp(kappa * torch.cos(angle - centers) + torch.log(weights + 1e-12), dim=0)


def chain_loss(geo32, raw, R_occs, t_occs, prior=None, lam=0.0, wR=1.0, wt=0.1):
    """The closure's loss (bpe.py:536-558) for one chain: geo32 (r, 9) float32 in the device
    layout {N:CA, CA:C, tau, 0C:1N, CA:C:1N, C:1N:1CA, psi, omega, phi} per residue."""
    import torch
    r = geo32.shape[0]
    om, th, ph = (wrap(x) for x in raw.unbind(-1))
    n0, ca0, c0 = _start(float(geo32[0, 1]), float(geo32[0, 0]), float(geo32[0, 2]))
    xyz = [torch.tensor(v) for v in (n0, ca0, c0)]
    # NERFBuilder's dihedral table (nerf.py:91-100): psi, omega, phi per junction
    nan = torch.tensor([np.nan])
    psi = torch.cat((geo32[:r - 1, 6], nan))[:-1]
    omega = torch.cat((om, nan))[:-1]
    phi = torch.cat((nan, ph))[1:]
    dih = torch.stack([psi, omega, phi]).T
    for i in range(r - 1):
        xyz.append(_place(xyz[-3], xyz[-2], xyz[-1], geo32[i, 4], geo32[i, 3], dih[i][0]))
        xyz.append(_place(xyz[-3], xyz[-2], xyz[-1], th[i], geo32[i + 1, 0], dih[i][1]))
        xyz.append(_place(xyz[-3], xyz[-2], xyz[-1], geo32[i + 1, 2], geo32[i + 1, 1], dih[i][2]))
    coords = torch.stack(xyz)
    frames = [_frame(*coords[3 * i:3 * (i + 1)]) for i in range(1, r)]
    rot = sum(0.5 * torch.sum((Ro - Rn) ** 2) for (Rn, _), Ro in zip(frames, R_occs))
    trans = sum(torch.sum((to - tn) ** 2) for (_, tn), to in zip(frames, t_occs))
    loss = wR * rot + wt * trans
    if lam > 0.0:
        (c_o, w_o), (c_t, w_t), (c_p, w_p) = prior
        p = sum(circ_kde_prior(o, c_o, w_o, 50.) + circ_kde_prior(t, c_t, w_t, 20.) + circ_kde_prior(f, c_p, w_p, 20.)
                for o, t, f in zip(om, th, ph))
        loss = loss + lam * p
    return loss


def optimize(geo, x0, R_occs, t_occs, prior=None, lam=0.0):
    """optimize_glues_entry_torch (ret_all) up to snapping: the wrapped optimum (r-1, 3),
    the LBFGS iteration / evaluation counts and the first / last loss."""
    import torch
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
        loss = chain_loss(geo32, raw, R, T, pr, lam)
        loss.backward()
        losses.append(loss.item())
        return loss

    opt.step(closure)
    st = opt.state[raw]
    return wrap(raw.detach()).numpy(), int(st["n_iter"]), int(st["func_evals"]), losses[0], losses[-1]


def snap_bin(arr, x):
    """snap_bin (bpe.py:495-524): the edge below / above the range, else the centre of the bin
    whose right edge is the first one above x (comparisons in float32, as on the tensor)."""
    x = np.float32(x)
    if x < np.float32(arr[0][0]):
        return arr[0][0]
    if x >= np.float32(arr[-1][1]):
        return arr[-1][1]
    i = bisect.bisect_right([np.float32(b) for _, b in arr], x)
    return sum(arr[i]) / 2
