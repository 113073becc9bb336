"""Embedding-table shard and wide & deep ops (GPU: csrc/hip/embedding.hip; CPU: the
same math in PyTorch, which is the numerics reference).

``EmbeddingShard``: one rank's share of a ``[num_features, D]`` embedding table
plus a wide (linear) weight per key. The scalar KV table (32-B slots with the
wide weight and its FTRL state, ``ops.kv_table``) is the key index; the bf16
row of a key lives at the SAME slot index of ``rows [capacity, D]``, next to a
row-wise AdaGrad accumulator and a first-touch init flag.
"""
from __future__ import annotations

import math

import torch

from .kv_table import EMPTY_KEY, KVTable, UpdateRule
from .native import hipops, is_gpu


class EmbeddingShard:
    def __init__(self, capacity: int, dim: int, device="cpu", *, init_scale: float = 0.01,
                 seed: int = 0):
        self.table = KVTable(capacity, device)
        cap = self.table.capacity
        self.capacity, self.dim = cap, dim
        self.device = torch.device(device)
        self.rows = torch.zeros(cap, dim, dtype=torch.bfloat16, device=self.device)
        self.acc = torch.zeros(cap, dtype=torch.float32, device=self.device)
        self.inited = torch.zeros(cap, dtype=torch.uint8, device=self.device)
        self.init_scale, self.seed = float(init_scale), int(seed)
        self.gpu = self.device.type == "cuda"

    def nbytes(self) -> int:
        return self.table.nbytes() + self.capacity * (self.dim * 2 + 4 + 1)

    # -------------------------------------------------------------- checkpoint
    def state(self) -> dict:
        """Every occupied slot: mixed key, wide state (w, z, n), bf16 row, row AdaGrad
        accumulator (device tensors, one entry per key)."""
        mk, w, z, n = self.table.occupied()
        mask = self.table.slots[:, 0] != EMPTY_KEY
        # cnt | flags word: the update count a decaying SGD wide rule reads
        return {"mkeys": mk, "w": w, "z": z, "n": n, "rows": self.rows[mask],
                "acc": self.acc[mask], "cnt": self.table.slots[mask, 3]}

    def load_state(self, mkeys, w, z, n, rows, acc, cnt=None) -> torch.Tensor:
        """Insert keys with their saved state (rows are marked initialised)."""
        slot = self.table.load(mkeys, w, z, n)
        self.rows[slot] = rows.to(self.device, torch.bfloat16)
        self.acc[slot] = acc.to(self.device, torch.float32)
        if cnt is not None:
            self.table.slots[slot, 3] = cnt.to(self.device, torch.int64)
        self.inited[slot] = 1
        return slot

    # -------------------------------------------------------------- pull side
    def resolve(self, mkeys: torch.Tensor, n_dev=None, slot=None, w=None):
        """Lookup-or-insert mixed keys; first-touch rows are initialised N(0, scale)
        deterministically from the key. Returns (slot int64, wide weight f32)."""
        if self.gpu:
            it, iv, isd, seed = self.table.init.args()
            n = mkeys.numel()
            slot = torch.empty(n, dtype=torch.int64, device=self.device) if slot is None else slot
            w = torch.empty(n, dtype=torch.float32, device=self.device) if w is None else w
            H = hipops()
            H.kv_resolve(self.table.slots, mkeys, n_dev, slot, w, True, it, iv, isd, seed,
                         self.table._err, self.table._inserted, self.table.home_base,
                         self.table.home_m)
            H.emb_init_rows(slot, mkeys, n_dev, self.rows, self.inited, self.seed,
                            self.init_scale)
            return slot, w
        slot, w = self.table.resolve(mkeys, insert=True)
        new = torch.nonzero(self.inited[slot] == 0).flatten()
        if new.numel():
            s = slot[new]
            self.rows[s] = init_rows(mkeys[new], self.dim, self.seed, self.init_scale)
            self.inited[s] = 1
        return slot, w

    def gather_rows(self, slot: torch.Tensor) -> torch.Tensor:
        out = torch.empty(slot.numel(), self.dim, dtype=torch.bfloat16, device=self.device)
        if self.gpu:
            hipops().emb_gather_rows(slot, self.rows, out)
            return out
        out.copy_(self.rows[slot])
        return out

    # -------------------------------------------------------------- push side
    def update_rows(self, slot, grad=None, grad16=None, lr: float = 0.01, eps: float = 1e-8,
                    n_dev=None):
        """Row-wise AdaGrad; ``slot`` must be unique within one call."""
        if self.gpu:
            hipops().emb_update(slot, n_dev, grad, grad16, self.rows, self.acc, lr, eps)
            return
        n = slot.numel() if n_dev is None else int(n_dev.item())
        s = slot[:n]
        g = (grad if grad is not None else grad16.float())[:n].reshape(n, self.dim)
        a = self.acc[s] + (g * g).mean(1)
        self.acc[s] = a
        step = lr / (torch.sqrt(a) + eps)
        self.rows[s] = (self.rows[s].float() - step[:, None] * g).to(torch.bfloat16)

    def update_wide(self, slot, grad, rule: UpdateRule, stats, n_dev=None):
        self.table.update(slot, grad, rule, stats, n_dev=n_dev)


def _rng64(seed, idx):
    """splitmix64 of (seed, idx) — common.cuh rng64, vectorised in uint64 numpy."""
    import numpy as np

    with np.errstate(over="ignore"):
        z = seed + np.uint64(0x9E3779B97F4A7C15) * (idx + np.uint64(1))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def init_rows(mkeys: torch.Tensor, D: int, seed: int, scale: float) -> torch.Tensor:
    """Deterministic first-touch rows: Box-Muller on rng64(seed ^ key, d) — the same
    stream as the emb_init_rows kernel."""
    import numpy as np

    k = mkeys.cpu().numpy().view(np.uint64)[:, None]
    d = np.arange(D, dtype=np.uint64)[None, :]
    r = _rng64(np.uint64(seed) ^ k, d)
    u1 = ((r >> np.uint64(40)) + np.uint64(1)).astype(np.float32) * np.float32(1.0 / 16777217.0)
    u2 = ((r >> np.uint64(16)) & np.uint64(0xFFFFFF)).astype(np.float32) * np.float32(
        1.0 / 16777216.0)
    z = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)
    return torch.from_numpy((z * scale).astype(np.float32)).to(torch.bfloat16).to(mkeys.device)


def expand(local_col: torch.Tensor, nnz: int, src: torch.Tensor, idx=None, out=None):
    """X0[p] = src[idx[local_col[p]]] (or src[local_col[p]]): the [B*S, D] MLP input."""
    D = src.shape[1]
    if out is None:
        out = torch.empty(nnz, D, dtype=torch.bfloat16, device=src.device)
    if is_gpu(src):
        hipops().emb_expand(local_col, nnz, idx, src, out)
        return out
    r = local_col[:nnz].long()
    if idx is not None:
        r = idx[r]
    out[:nnz] = src[r]
    return out


_WIDE_OK: dict[int, bool] = {}


def grad_wide_fused(D: int, gpu: bool) -> bool:
    """Whether ``grad_reduce`` can produce the wide gradient in the same pass."""
    if not gpu:
        return False
    ok = _WIDE_OK.get(D)
    if ok is None:  # (asked once per D: a native call per step is host issue time)
        ok = _WIDE_OK[D] = bool(hipops().emb_grad_wide_ok(D))
    return ok


def grad_reduce(loc, dX0: torch.Tensor, D: int, u_cap: int, out=None, coef=None, width: int = 0,
                g_wide=None):
    """dE[u] = sum of dX0 rows over u's occurrences (fp32 [u_cap, D]). With ``g_wide``
    (GPU, ``grad_wide_fused``): also g_wide[u] = sum of coef[row] over u's occurrences
    (row = position // width, the wide part's gradient), in the same pass."""
    nnz = loc.nnz
    if out is None:
        out = torch.empty(u_cap, D, dtype=torch.float32, device=dX0.device)
    if is_gpu(dX0):
        hipops().emb_grad_reduce(loc.pos_s, loc.segid, loc.seg_start, loc.n_uniq, u_cap, nnz, dX0,
                                 D, out, coef, width, g_wide)
        return out
    out.zero_()
    seg = loc.segid[:nnz].long() - 1  # segid is 1-based in the localiser
    out.index_add_(0, seg, dX0.reshape(-1, D)[loc.pos_s[:nnz].long()].float())
    return out


def head(h, w, b, wide_w, local_col, S: int, labels, coef, dh, dw, db, metrics, hist,
         nbins: int, db_h=None):
    """Deep logit + wide margin, logistic loss, metrics, AUC histogram, head grads;
    ``db_h`` (optional) += column sums of ``dh`` (bias gradient of the last hidden
    layer, computed as w * sum_r coef_r [h > 0] without re-reading dh)."""
    if is_gpu(h):
        hipops().wd_head(h, w, b, wide_w, local_col, S, labels, coef, dh, dw, db, metrics, hist,
                         nbins, db_h)
        return
    B, H = h.shape
    hf = h.float()
    m = hf @ w + b[0]
    lc = local_col[:B * S].long().reshape(B, S)
    m = m + wide_w[lc].sum(1)
    y = torch.where(labels[:B] > 0, 1.0, -1.0)
    ym = y * m
    loss = torch.nn.functional.softplus(-ym)
    c = -y * torch.sigmoid(-ym)
    coef[:B] = c
    dh.copy_((c[:, None] * w[None, :] * (hf > 0)).to(torch.bfloat16))
    dw += (c[:, None] * hf).sum(0)
    db += c.sum()
    if db_h is not None:
        db_h += w * (c[:, None] * (hf > 0)).sum(0)
    metrics[0] += loss.double().sum()
    metrics[1] += ((y > 0) == (m > 0)).double().sum()
    metrics[2] += B
    p = torch.sigmoid(m)
    pb = torch.clamp((p * nbins).long(), 0, nbins - 1)
    hist += torch.bincount(pb + torch.where(y > 0, nbins, 0), minlength=2 * nbins).to(hist.dtype)


def colsum(x: torch.Tensor, out: torch.Tensor, accumulate: bool = False):
    """out (+)= column sums of x [B, N] (bf16) in fp32."""
    if is_gpu(x):
        if not accumulate:
            out.zero_()
        hipops().colsum_bf16(x, out)
        return out
    if accumulate:
        out += x.float().sum(0)
    else:
        out.copy_(x.float().sum(0))
    return out


def adam(p, g, m, v, *, lr, step: int, b1=0.9, b2=0.999, eps=1e-8, gscale=1.0, p16=None,
         step_dev=None, zero_grad: bool = False):
    """Adam on fp32 master weights (+ bf16 copy ``p16``). ``step_dev`` (GPU): int64 device
    step clock holding the steps completed so far; the kernel takes its bias corrections
    from it (step = step_dev + 1), so the update can be replayed from a HIP graph.
    ``zero_grad``: g is zeroed once read (the next step accumulates into it)."""
    if is_gpu(p):
        hipops().adam_update(p, g, m, v, lr, b1, b2, eps, step, gscale, p16, step_dev,
                             bool(zero_grad))
        return
    gs = g * gscale
    m.mul_(b1).add_((1 - b1) * gs)
    v.mul_(b2).add_((1 - b2) * gs * gs)
    p.sub_(lr * (m / (1 - b1 ** step)) / (torch.sqrt(v / (1 - b2 ** step)) + eps))
    if p16 is not None:
        p16.copy_(p.to(torch.bfloat16))
    if zero_grad:
        g.zero_()


def xavier(n_out: int, n_in: int, gen: torch.Generator) -> torch.Tensor:
    a = math.sqrt(6.0 / (n_in + n_out))
    return (torch.rand(n_out, n_in, generator=gen) * 2 - 1) * a
