"""Sparse linear-model forward / backward on localized minibatches.

GPU: ``linear_fwd`` (Xw + loss + dL/dXw + accuracy + AUC histogram in one
launch) and ``linear_bwd`` (segmented reduction in CSC order), see
csrc/hip/linear.hip. CPU: the same math with plain PyTorch ops, which is also the
fp32 reference the HIP kernels are tested against.

Loss types follow the reference ``LossConfig`` enum
(src/app/linear_method/proto/linear.proto: SQUARE=1, LOGIT=2, HINGE=3,
SQUARE_HINGE=4); labels are +1 / -1 (>0 is positive).
"""
from __future__ import annotations

import torch

from .native import hipops, is_gpu

LOSS_TYPES = {"square": 1, "logit": 2, "hinge": 3, "square_hinge": 4}
AUC_BINS = 2048

# Striped float64 accumulators for the per-step loss / accuracy / optimizer stats
# (csrc/hip/common.cuh acc_stripe): kernels add into stripe blockIdx % 64 (one
# 128-B line each) instead of one contended address; logical slot k = the sum of
# element k over the stripes. CPU code adds into stripe 0.
ACC_STRIPES, ACC_STRIDE = 64, 16
HIST_STRIPES = 8  # AUC histogram copies (linear_fwd flushes block b into stripe b % 8)


def new_accum(device) -> torch.Tensor:
    return torch.zeros(ACC_STRIPES * ACC_STRIDE, dtype=torch.float64, device=device)


def accum_total(t: torch.Tensor) -> torch.Tensor:
    """Logical [16] view of a striped accumulator (a small tensor is returned as is)."""
    if t.numel() >= ACC_STRIPES * ACC_STRIDE:
        return t.view(-1, ACC_STRIDE).sum(0)
    return t


def loss_id(loss) -> int:
    return loss if isinstance(loss, int) else LOSS_TYPES[str(loss).lower()]


def _rows_of(B: int, width: int, row_ptr, device):
    if row_ptr is None:
        return torch.arange(B, device=device).repeat_interleave(width)
    counts = row_ptr[1:] - row_ptr[:-1]
    return torch.repeat_interleave(torch.arange(B, device=device), counts)


def loss_terms_torch(m: torch.Tensor, labels: torch.Tensor, loss: int):
    """(loss, coef = dL/dm, coef2 = d2L/dm2) elementwise, fp32."""
    y = torch.where(labels > 0, 1.0, -1.0).to(m.dtype)
    ym = y * m
    if loss == 1:
        d = m - labels
        return 0.5 * d * d, d, torch.ones_like(m)
    if loss == 3:
        return torch.clamp(1 - ym, min=0), torch.where(ym < 1, -y, torch.zeros_like(y)), torch.zeros_like(m)
    if loss == 4:
        h = torch.clamp(1 - ym, min=0)
        return h * h, -2 * y * h, torch.where(ym < 1, 2.0, 0.0).to(m.dtype)
    tau = torch.sigmoid(-ym)
    return torch.nn.functional.softplus(-ym), -y * tau, tau * (1 - tau)


def linear_forward(local_col, w_local, labels, *, B: int, width: int = 0, row_ptr=None,
                   vals=None, loss="logit", xw=None, coef=None, coef2=None, metrics=None,
                   hist=None):
    """Returns (xw, coef, coef2). ``metrics`` (float64[>=5]) += [loss, correct, n, ...];
    ``hist`` (int32[2*AUC_BINS]) accumulates the bucketed-AUC histogram."""
    L = loss_id(loss)
    dev = local_col.device
    if is_gpu(local_col):
        coef = torch.empty(B, dtype=torch.float32, device=dev) if coef is None else coef
        hipops().linear_fwd(row_ptr, B, width, local_col, vals, w_local, labels, L, xw, coef,
                            coef2, metrics, hist, AUC_BINS)
        return xw, coef, coef2
    rows = _rows_of(B, width, row_ptr, dev)
    col = local_col.long()
    valid = col >= 0
    contrib = torch.where(valid, w_local[col.clamp(min=0)], torch.zeros((), device=dev))
    if vals is not None:
        contrib = contrib * vals
    m = torch.zeros(B, dtype=torch.float32, device=dev).index_add_(0, rows, contrib.float())
    lo, c, c2 = loss_terms_torch(m, labels[:B].float(), L)
    if xw is not None:
        xw.copy_(m)
    if coef is not None:
        coef.copy_(c)
    else:
        coef = c
    if coef2 is not None:
        coef2.copy_(c2)
    if metrics is not None:
        y = torch.where(labels[:B] > 0, 1.0, -1.0)
        metrics[0] += float(lo.double().sum())
        metrics[1] += float(((y > 0) == (m > 0)).double().sum())
        metrics[2] += float(B)
    if hist is not None:
        p = torch.sigmoid(m)
        b = torch.clamp((p * AUC_BINS).long(), 0, AUC_BINS - 1)
        off = torch.where(labels[:B] > 0, AUC_BINS, 0)
        hist[:2 * AUC_BINS] += torch.bincount(b + off, minlength=2 * AUC_BINS).to(hist.dtype)
    return (xw if xw is not None else m), coef, (coef2 if coef2 is not None else c2)


def linear_backward(loc, coef, *, B: int, width: int = 0, rows=None, vals=None, coef2=None):
    """grad[u] (and hess[u] if coef2 given) into loc.grad / loc.hess."""
    if getattr(loc, "tile", None) is not None:  # tile-deduplicated ("tp") localisation
        t = loc.tile
        hipops().tp_backward(t.rep, t.dcnt, loc.nnz, rows, width, vals, coef, t.psum, loc.pos_s,
                             loc.segid, t.n_ent, loc.grad)
        return loc.grad, None
    if is_gpu(coef):
        hipops().linear_bwd(loc.pos_s, loc.segid, loc.nnz, rows, width, vals, coef,
                            coef2 if loc.hess is not None else None, loc.grad,
                            loc.hess if coef2 is not None else None)
        return loc.grad, loc.hess
    dev = coef.device
    if rows is None:
        rows = torch.arange(B, device=dev).repeat_interleave(width) if width else None
    r = rows.long()
    x = vals.float() if vals is not None else torch.ones(r.numel(), device=dev)
    col = loc.local_col.long()
    U = loc.grad.numel()
    g = torch.zeros(U, dtype=torch.float32, device=dev).index_add_(0, col, coef[r] * x)
    loc.grad.copy_(g)
    if coef2 is not None and loc.hess is not None:
        h = torch.zeros(U, dtype=torch.float32, device=dev).index_add_(0, col, coef2[r] * x * x)
        loc.hess.copy_(h)
    return loc.grad, loc.hess


_FB_WIDTHS: dict[int, bool] = {}  # width -> tp_fwd_bwd has a kernel instance for it


def _tp_fused(loc, w_local, B, width, row_ptr, rows) -> bool:
    t = getattr(loc, "tile", None)
    if not (t is not None and t.ent_uid is not None and row_ptr is None and rows is None
            and bool(width) and loc.nnz == B * width and is_gpu(w_local)):
        return False
    ok = _FB_WIDTHS.get(width)
    if ok is None:  # (asked once per width: a native call per step is host issue time)
        ok = _FB_WIDTHS[width] = bool(hipops().tp_fwd_bwd_supported(width))
    return ok


def linear_fwd_bwd(loc, w_local, labels, *, B: int, width: int = 0, row_ptr=None, rows=None,
                   vals=None, loss="logit", coef=None, metrics=None, hist=None, update=None):
    """Forward (loss, dL/dm, metrics, AUC histogram) and backward into loc.grad of one
    minibatch; returns (coef, grad). A fixed-width "tp" localisation runs ONE fused
    per-tile kernel plus the entry scan (tploc.hip tp_fwd_bwd: no per-occurrence
    local-column gather, no coef round trip through memory); anything else runs
    linear_forward + linear_backward.

    ``update = (slots, slot_idx, rule, stats, step_counter)`` (tp path only): the entry
    scan also applies the optimizer update to every key's slot and folds the step's
    AUC epilogue (tp_seg_update: no grad round trip, one launch less); returns
    (coef, None). Check ``fused_update_ok`` first."""
    if _tp_fused(loc, w_local, B, width, row_ptr, rows):
        t = loc.tile
        coef = torch.empty(B, dtype=torch.float32, device=w_local.device) if coef is None else coef
        hipops().tp_fwd_bwd(t.rep, t.dcnt, t.ent_uid, loc.nnz, width, vals, w_local, labels, B,
                            loss_id(loss), coef, metrics, hist, AUC_BINS, t.psum, loc.pos_s,
                            loc.segid, t.n_ent, loc.grad, update is None)
        if update is not None:
            slots, slot_idx, rule, stats, step_counter = update
            hipops().tp_seg_update(loc.pos_s, loc.segid, loc.nnz, t.n_ent, t.psum, loc.seg_start,
                                   loc.n_uniq, t.pieces, slot_idx, slots, *rule.args(), stats,
                                   hist, metrics, step_counter)
            return coef, None
        return coef, loc.grad
    if update is not None:
        raise ValueError("a fused update needs the tp forward/backward (fused_update_ok)")
    from .localize import ensure_local_col

    _, coef, _ = linear_forward(ensure_local_col(loc), w_local, labels, B=B, width=width,
                                row_ptr=row_ptr, vals=vals, loss=loss, coef=coef,
                                metrics=metrics, hist=hist)
    grad, _ = linear_backward(loc, coef, B=B, width=width, rows=rows, vals=vals)
    return coef, grad


def fused_update_ok(loc, w_local, *, B: int, width: int = 0, row_ptr=None, rows=None,
                    vals=None) -> bool:
    """Can ``linear_fwd_bwd(..., update=...)`` run (tp localisation with its (sum, count)
    accumulators, fixed width, binary features: |gradient| <= B < 2^25, GPU)?"""
    return (vals is None and B < (1 << 25) and _tp_fused(loc, w_local, B, width, row_ptr, rows)
            and getattr(loc.tile, "pieces", None) is not None)


def auc_from_hist(hist: torch.Tensor, metrics: torch.Tensor, step_counter=None):
    """metrics[3] += AUC of the histogram, metrics[4] += 1; zeroes hist; optionally
    increments a device step counter (one epilogue kernel per step)."""
    if is_gpu(hist):
        hipops().auc_from_hist(hist, AUC_BINS, metrics, step_counter)
        return
    h = hist.view(-1, 2 * AUC_BINS).sum(0)  # stripes (CPU code only writes stripe 0)
    neg = h[:AUC_BINS].double()
    pos = h[AUC_BINS:].double()
    P, N = float(pos.sum()), float(neg.sum())
    if P > 0 and N > 0:
        below = torch.cumsum(neg, 0) - neg
        area = float((pos * (below + 0.5 * neg)).sum())
        metrics[3] += area / (P * N)
        metrics[4] += 1
    hist.zero_()
    if step_counter is not None:
        step_counter += 1


def exact_auc(scores: torch.Tensor, labels: torch.Tensor) -> float:
    """Exact ROC AUC by sorting (reference Evaluation::auc, src/util/evaluation.h:22-45)."""
    s = scores.double().cpu()
    y = labels.cpu() > 0
    order = torch.argsort(s)
    ranks = torch.empty_like(s)
    # average ranks for ties
    ss = s[order]
    uniq, inv, cnt = torch.unique_consecutive(ss, return_inverse=True, return_counts=True)
    ends = torch.cumsum(cnt, 0).double()
    avg = ends - (cnt.double() - 1) / 2
    ranks[order] = avg[inv]
    P = int(y.sum())
    N = y.numel() - P
    if P == 0 or N == 0:
        return float("nan")
    return float((ranks[y].sum() - P * (P + 1) / 2) / (P * N))
