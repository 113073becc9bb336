"""Darlin block-coordinate-descent ops (L1 logistic regression).

GPU: ``csrc/hip/bcd.hip`` (K11 block gradient, K13 coordinate update with KKT
filter + trust region, K12 margin update, objective / server statistics).
CPU: the same math in plain fp64 PyTorch, which is both the host path of the
runtime apps and the reference the HIP kernels are tested against.

Conventions (shared with the kernels):
* a rank's training matrix is ONE CSC over the global column space: ``col`` and
  ``row`` int32 per nnz sorted by column, ``val`` f32 per nnz or ``None``
  (binary). A feature block is a column range ``[c0, c0+ncols)`` stored in the
  nnz range ``[p0, p1)``.
* ``ym`` (fp64, per row) is the margin ``y_i * x_i.w``; the reference keeps
  ``dual_i = exp(ym_i)`` instead (src/app/linear_method/darlin.h:288-293) and
  uses ``tau_i = 1 / (1 + dual_i)``.
* ``w``, ``delta`` (fp64) and ``active`` (uint8) are indexed by global column.

Reference math: gradient darlin.h:381-427, update darlin.h:206-246, dual update
darlin.h:472-502, objective darlin.h:504-511, server evaluate darlin.h:248-265.
"""
from __future__ import annotations

import numpy as np
import torch

from .native import hipops, is_gpu


HOT_BIT = 1 << 62


SKIP_BIT = 1 << 61


def build_chunks(colptr, c0: int, c1: int, small: int = 64, hot: int = 4096,
                 skip=None) -> np.ndarray:
    """Load-balanced work list of the CSC columns [c0, c1) for ``grad``'s chunked
    kernel: int64 entry offsets (+ end sentinel); columns of <= ``small`` entries
    are packed whole into chunks of <= ``small`` entries, longer ("hot") columns
    are cut into pieces of <= ``hot`` entries flagged with HOT_BIT. ``skip`` (bool
    per column of the block): columns another kernel sums (the row pass's LDS hot
    columns) become one chunk each flagged with SKIP_BIT, which the kernel passes over."""
    cp = np.asarray(colptr, dtype=np.int64)
    n = np.diff(cp[c0:c1 + 1])
    out = []
    cur, cur_len = -1, 0
    for j in np.flatnonzero(n):
        a, m = int(cp[c0 + j]), int(n[j])
        if skip is not None and skip[j]:
            if cur >= 0:
                out.append(cur)
                cur = -1
            out.append(a | SKIP_BIT)
            continue
        if m > small:
            if cur >= 0:
                out.append(cur)
                cur = -1
            out.extend(p | HOT_BIT for p in range(a, a + m, hot))
            continue
        if cur < 0 or cur_len + m > small:
            if cur >= 0:
                out.append(cur)
            cur, cur_len = a, 0
        cur_len += m
    if cur >= 0:
        out.append(cur)
    out.append(int(cp[c1]))
    ch = np.asarray(out, dtype=np.int64)
    pos = ch & ~(HOT_BIT | SKIP_BIT)
    assert np.all(np.diff(pos) > 0) and pos[0] >= cp[c0] and pos[-1] == cp[c1]
    return ch


def grad(col, row, val, p0: int, p1: int, c0: int, ncols: int, ym, y, delta, active,
         G=None, U=None, chunks=None, zeroed: bool = False, rowq=None, rowq_ready: bool = False,
         urows=None):
    """Block gradient: returns (G, U) fp64[ncols] (inactive columns contribute 0).
    ``chunks`` (device int64 from ``build_chunks``) selects the load-balanced kernel;
    ``rowq`` (fp64 [2 * rows] scratch, with ``chunks``): the per-example factors are
    packed first so each entry gathers one 16-B record (wide blocks);
    ``zeroed``: G / U already hold zeros (left by ``update(consume=True)``);
    ``rowq_ready``: ``rowq`` already holds the factors of the block's examples (a
    ``rowpass`` wrote them), so the packing pass is skipped; ``urows`` (device int32, the
    block's distinct examples): the packing covers only them instead of every example."""
    dev = ym.device
    if G is None:
        G = torch.empty(ncols, dtype=torch.float64, device=dev)
    if U is None:
        U = torch.empty(ncols, dtype=torch.float64, device=dev)
    if is_gpu(ym):
        if chunks is not None:
            hipops().bcd_grad_chunked(col, row, val, chunks, c0, ncols, ym, y, delta, active,
                                      G, U, zeroed, rowq, bool(rowq_ready), urows)
        else:
            hipops().bcd_grad(col, row, val, p0, p1, c0, ncols, ym, y, delta, active, G, U)
        return G, U
    G.zero_()
    U.zero_()
    c = col[p0:p1].long() - c0
    r = row[p0:p1].long()
    keep = active[c0 + c].bool()
    c, r = c[keep], r[keep]
    tau = 1.0 / (1.0 + torch.exp(ym[r]))
    yr = y[r].double()
    t2 = tau * (1 - tau)
    dl = delta[c0 + c]
    if val is None:
        g = -yr * tau
        u = torch.clamp(t2 * torch.exp(dl), max=0.25)
    else:
        v = val[p0:p1][keep].double()
        g = -yr * tau * v
        u = torch.clamp(t2 * torch.exp(v.abs() * dl), max=0.25) * v * v
    G.index_add_(0, c, g)
    U.index_add_(0, c, u)
    return G, U


def grad_rows(col_r, row_r, val_r, p0: int, p1: int, c0: int, ncols: int, ym, y, delta,
              active, G, U, part, W: int, k2: int, upd: dict | None = None):
    """Block gradient of a NARROW block (ncols <= ``hipops().bcd_rows_max_cols()``) from
    the row-sorted entries: sequential per-row reads, LDS fixed-point column sums at
    scale 2^k2 (``fixed_point_shift`` of the block's entry count), W workgroup partials
    in ``part`` reduced in a
    fixed order (deterministic). Same result as ``grad`` up to the 2^-k2 quantisation.
    ``upd`` (GPU, one rank): ``dict(w, dw, vio, counter, eta, lam, delta_max, kkt_thr)``:
    the coordinate update (``update``'s arithmetic) runs in the kernel's last workgroup and
    writes ``dw``; ``part`` is then the block's zeroed 2 x ncols int64 accumulator and
    G / U are not written."""
    if is_gpu(ym):
        u = upd or {}
        hipops().bcd_grad_rows(col_r, row_r, val_r, p0, p1, c0, ncols, ym, y, delta, active,
                               int(k2), int(W), part, G, U, u.get("w"), u.get("dw"),
                               u.get("vio"), u.get("counter"), float(u.get("eta", 1.0)),
                               float(u.get("lam", 0.0)), float(u.get("delta_max", 0.0)),
                               float(u.get("kkt_thr", 0.0)))
        return G, U
    return grad(col_r, row_r, val_r, p0, p1, c0, ncols, ym, y, delta, active, G, U)


def dense_rows(row_r, col_r, val_r, p0: int, p1: int, c0: int, rows: int):
    """Dense per-example layout of a block with at most one entry per example:
    (dcol int32 [rows]: the entry's column relative to c0, -1 = none; dval float32
    [rows] or None). 4 B per example, read in example order by ``rowpass``."""
    dev = row_r.device
    dcol = torch.full((rows,), -1, dtype=torch.int32, device=dev)
    dval = None if val_r is None else torch.zeros(rows, dtype=torch.float32, device=dev)
    if p1 > p0:
        r = row_r[p0:p1].long()
        dcol[r] = (col_r[p0:p1].long() - c0).to(torch.int32)
        if dval is not None:
            dval[r] = val_r[p0:p1]
    return dcol, dval


def hot_layout(dcol, colptr, c0: int, c1: int, nhot: int = 2048, min_share: float = 0.5):
    """Hot / cold split of a WIDE block with a dense layout (``dense_rows``): its ``nhot``
    most frequent columns are summed in LDS by the row pass and the rest by the chunked
    column-order kernel. Returns None when the hot columns hold < ``min_share`` of the
    entries, else (kenc int32 [rows]: -2 - hot slot / the column (cold) / -1 none,
    hcols int32 [nhot] hot slot -> column, chunks of the cold columns (hot ones
    SKIP_BIT-flagged), hot entry count)."""
    cp = np.asarray(colptr, dtype=np.int64)
    cnt = np.diff(cp[c0:c1 + 1])
    ncols = c1 - c0
    if ncols <= nhot or cnt.sum() == 0:
        return None
    top = np.argpartition(-cnt, nhot - 1)[:nhot]
    hot_entries = int(cnt[top].sum())
    if hot_entries < min_share * cnt.sum():
        return None
    hcols = np.sort(top).astype(np.int32)
    assert hcols[0] >= 0 and hcols[-1] < ncols
    slot = torch.full((ncols,), -1, dtype=torch.int32)
    slot[torch.from_numpy(hcols).long()] = torch.arange(nhot, dtype=torch.int32)
    slot = slot.to(dcol.device)
    has = dcol >= 0
    hs = torch.where(has, slot[dcol.clamp_min(0).long()], torch.full_like(dcol, -1))
    kenc = torch.where(hs >= 0, -2 - hs, dcol)
    skip = np.zeros(ncols, dtype=bool)
    skip[hcols] = True
    chunks = build_chunks(cp, c0, c1, skip=skip)
    return kenc, torch.from_numpy(hcols).to(dcol.device), chunks, hot_entries


def rowpass(ym, y, delta, active, *, jcol=None, jval=None, jdw=None, jncols: int = 0,
            kcol=None, kval=None, c0: int = 0, ncols: int = 0, k2: int = 0, W: int = 1,
            part=None, G=None, U=None, rowq=None, hcols=None, part2=None, tau32: bool = False):
    """GPU row pass over dense block layouts (``dense_rows``): first the pending dual
    update of block j (``jcol`` / ``jval`` / its ``jdw``: ym_i += y_i dw_c x_ic), then on
    the updated margins block k's gradient: narrow (``part`` given: fixed-point column
    sums into ``G`` / ``U``, as ``grad_rows``) or the per-example factors of a wide block
    into ``rowq`` (for ``grad(..., rowq_ready=True)``); with ``hcols`` (``hot_layout``),
    a wide block's hot columns in LDS and the cold entries' factors into ``rowq``;
    ``part2`` (narrow): leave the segment sums there for ``update(..., part2=)`` instead
    of storing G / U. ``tau32``: tau_i = 1 / (1 + exp(ym_i)) in fp32 (the G / U sums
    stay fp64 / fixed point; ~1e-7 relative per factor), the fast mode of the benchmark.
    Equal to ``dual`` followed by ``grad_rows`` / the rowq packing up to the fixed-point
    quantisation (tests/test_darlin_gpu.py)."""
    hipops().bcd_rowpass(ym, y, jcol, jval, jdw, int(jncols), kcol, kval, int(c0), int(ncols),
                         delta, active, int(k2), int(W), part, G, U, rowq, hcols, part2, bool(tau32))


def fixed_point_shift(entries: int, max_abs_val: float) -> int:
    """k such that the sum of ALL of a block's ``entries`` addends (|g| <= |v|,
    |u| <= v^2 / 4) stays below 2^61 at scale 2^k (grad_rows: the per-workgroup
    partials and their reduction are exact int64 sums)."""
    import math

    bound = max(1.0, max_abs_val, 0.25 * max_abs_val * max_abs_val) * max(1, entries)
    return max(0, min(60, 61 - math.ceil(math.log2(bound))))


def update(c0: int, ncols: int, G, U, w, delta, active, eta: float, lam: float,
           delta_max: float, kkt_thr: float, dw=None, vio=None, consume: bool = False,
           nan_filtered: bool = False, part2=None, k2: int = 0):
    """Coordinate update of block [c0, c0+ncols). Returns (dw fp64[ncols], vio) where
    ``vio`` is an int64[1] tensor holding the max KKT violation as fp64 bits
    (max-accumulated across calls; see ``violation``). ``consume`` zeroes G / U
    after reading them. ``nan_filtered``: a KKT-filtered column's dw is NaN instead of
    0 (the reference server's mark, src/app/linear_method/darlin.h:228-231), for
    ``replica``. ``part2`` (GPU): G / U come from a narrow row pass's segment sums at
    fixed-point scale 2^k2 (``rowpass(..., part2=)``) instead of G / U."""
    dev = w.device
    if dw is None:
        dw = torch.empty(ncols, dtype=torch.float64, device=dev)
    if vio is None:
        vio = torch.zeros(1, dtype=torch.int64, device=dev)
    if is_gpu(w):
        hipops().bcd_update(c0, ncols, G, U, w, delta, active, dw, eta, lam, delta_max, kkt_thr,
                            vio, consume, nan_filtered, part2, int(k2))
        return dw, vio
    sl = slice(c0, c0 + ncols)
    act = active[sl].bool()
    g, u = G[:ncols], U[:ncols] / eta + 1e-10
    gp, gn = g + lam, g - lam
    wk = w[sl].clone()
    zero = wk == 0
    v = torch.zeros_like(g)
    v = torch.where(zero & (gp < 0), -gp, v)
    v = torch.where(zero & ~(gp < 0) & (gn > 0), gn, v)
    filt = zero & ~(gp < 0) & ~(gn > 0) & (gp > kkt_thr) & (gn < -kkt_thr) & act
    upd = act & ~filt
    d = -wk
    d = torch.where(gp <= u * wk, -gp / u, torch.where(gn >= u * wk, -gn / u, d))
    dk = delta[sl]
    d = torch.minimum(dk, torch.maximum(-dk, d))
    d = torch.where(upd, d, torch.zeros_like(d))
    delta[sl] = torch.where(upd, torch.clamp(2 * d.abs() + .1, max=delta_max), dk)
    w[sl] = wk + d
    active[sl] = torch.where(filt, torch.zeros_like(active[sl]), active[sl])
    dw[:ncols] = torch.where(filt, torch.full_like(d, float("nan")), d) if nan_filtered else d
    vm = float(torch.where(upd, v, torch.zeros_like(v)).max()) if ncols else 0.0
    cur = violation(vio)
    if vm > cur:
        vio.copy_(torch.tensor([vm], dtype=torch.float64).view(torch.int64))
    if consume:
        G[:ncols] = 0
        U[:ncols] = 0
    return dw, vio


def replica(c0: int, ncols: int, own0: int, own1: int, dw, w, delta, active, delta_max: float):
    """Replay the owners' coordinate updates of block [c0, c0+ncols) (all-gathered
    ``dw`` with NaN marks) on this rank's replica outside its own slice [own0, own1):
    NaN -> column leaves the active set, else (if active) w += d and the trust region
    becomes min(delta_max, 2|d| + .1), the owner's arithmetic exactly. NaN marks are
    then zeroed in ``dw`` (in place) for the dual update."""
    if is_gpu(w):
        hipops().bcd_replica(c0, ncols, own0, own1, dw, w, delta, active, delta_max)
        return dw
    d = dw[:ncols]
    nan = torch.isnan(d)
    j = torch.arange(ncols, device=d.device)
    other = (j < own0) | (j >= own1)
    sl = slice(c0, c0 + ncols)
    act = active[sl].bool()
    upd = other & ~nan & act
    delta[sl] = torch.where(upd, torch.clamp(2 * d.abs() + .1, max=delta_max), delta[sl])
    w[sl] = torch.where(upd, w[sl] + d, w[sl])
    active[sl] = torch.where(other & nan, torch.zeros_like(active[sl]), active[sl])
    d[nan] = 0
    return dw


def violation(vio) -> float:
    """fp64 value of the violation accumulator written by ``update``."""
    return float(vio.detach().cpu().view(torch.float64)[0])


def dual(col, row, val, p0: int, p1: int, c0: int, ncols: int, dw, y, ym,
         unique_rows: bool = False):
    """ym_i += y_i * dw_c * x_ic over the block (in place). ``unique_rows``: no row
    occurs twice in [p0, p1) (GPU: plain read-modify-write instead of atomics)."""
    if is_gpu(ym):
        hipops().bcd_dual(col, row, val, p0, p1, c0, ncols, dw, y, ym, bool(unique_rows))
        return ym
    c = col[p0:p1].long() - c0
    r = row[p0:p1].long()
    d = dw[c]
    x = torch.ones_like(d) if val is None else val[p0:p1].double()
    ym.index_add_(0, r, y[r].double() * d * x)
    return ym


def objective(ym) -> torch.Tensor:
    """fp64[1] tensor: sum_i log(1 + exp(-ym_i)) (stays on device)."""
    out = torch.zeros(1, dtype=torch.float64, device=ym.device)
    if is_gpu(ym):
        hipops().bcd_objective(ym, out)
        return out
    out[0] = torch.nn.functional.softplus(-ym).sum()
    return out


def server_stats(w, active, c0: int, c1: int) -> torch.Tensor:
    """fp64[3] tensor: [sum |w| over nonzero, nnz(w), |active set|] over [c0, c1)."""
    out = torch.zeros(3, dtype=torch.float64, device=w.device)
    if is_gpu(w):
        hipops().bcd_server_stats(w, active, c0, c1, out)
        return out
    ws = w[c0:c1]
    nz = (ws != 0) & ~torch.isnan(ws)
    out[0] = ws[nz].abs().sum()
    out[1] = nz.sum()
    out[2] = active[c0:c1].double().sum()
    return out
