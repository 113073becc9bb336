"""Minibatch key localisation: unique keys + local column ids + CSC order.

Reference: ``Localizer::countUniqIndex`` / ``remapIndex`` (src/util/localizer.h:69-191)
which sort (key, pos) pairs on the CPU and rebuild a CSR with uint32 columns.
On the GPU (``csrc/hip/localize.hip``): mix -> radix sort over ``bits`` key bits ->
run-length encode, all into a preallocated workspace so a training step can be
captured into a HIP graph (the unique count stays on the device).

Outputs (``Localized``):
  uniq[0:U]      sorted unique *mixed* keys (grouped by owner shard)
  seg_start[0:U+1] start of each key's run in the sorted order
  pos_s[0:nnz]   nnz index of each element in key-sorted (= CSC) order
  segid[0:nnz]   1-based run id of each sorted element
  local_col[0:nnz] local column (run id) of every nnz in original (CSR) order
  n_uniq         int32[1] device counter U
  grad / hess    float[cap] buffers zeroed for the segments (backward targets)
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .keymix import mix, to_unsigned_order
from .native import hipops, is_gpu

TP_TILE = 8192  # occurrences per tp tile (csrc/hip/tploc.hip tp::kTile)


@dataclass
class Localized:
    uniq: torch.Tensor
    seg_start: torch.Tensor
    pos_s: torch.Tensor
    segid: torch.Tensor
    local_col: torch.Tensor
    n_uniq: torch.Tensor  # int32[1] (device)
    grad: torch.Tensor
    hess: torch.Tensor | None
    nnz: int
    # tile-deduplicated ("tp" mode): pos_s / segid / seg_start run over the
    # tile-distinct ENTRIES, not the nnz; the backward goes through tp_backward
    tile: object = None

    def num_unique(self) -> int:  # host sync
        return int(self.n_uniq.item())


@dataclass
class TileInfo:
    rep: torch.Tensor    # int16 [nnz] tile-local entry id of every position
    dcnt: torch.Tensor   # int32 [tiles] distinct keys per TP_TILE-key tile
    n_ent: torch.Tensor  # int32[1] total entries (device)
    psum: torch.Tensor   # float [tiles*TP_TILE] per-entry partial gradients (backward scratch)
    ent_uid: torch.Tensor | None = None  # int32 [tiles*TP_TILE] tile entry -> unique id
    cols_ready: bool = True  # False: local_col not materialised yet (ensure_local_col)
    pieces: torch.Tensor | None = None  # int64 [U] zeroed per localisation (tp_seg_update)


@dataclass
class FlatLoc:
    """A minibatch localised into the flat per-bucket layout (``Localizer(mode="tpf")``,
    csrc/hip/tploc.hip "tpf"; the 1-GPU fused step). Bucket workgroup b owns fixed
    regions: keys ``uniqf[b * key_region + unit * key_region / 2 + j]``, entries
    ``ent_pos`` (tile entry id) / ``ent_j`` (key index) at ``b * entry_region``, live
    counts ``cnt[b] = (D0, E0, D1, E1)``; ``slot_u`` receives each key's table slot at
    its pull and ``w_ent`` its weight in tile-entry order. There is no compact unique-key
    array: consumers run one workgroup per bucket (``tpf_step``). One object per
    workspace, refilled in place: ``gen`` counts its localisations (a pull issued ahead
    of the step is valid only for the generation it was issued for)."""
    rep: torch.Tensor       # int16 [nnz] tile entry of every position
    dcnt: torch.Tensor      # int32 [tiles] entries per tile
    psum: torch.Tensor      # float [tiles*TP_TILE] per-entry partial gradients
    w_ent: torch.Tensor     # float [tiles*TP_TILE] pulled weights in tile-entry order
    cnt: torch.Tensor
    uniqf: torch.Tensor
    ent_pos: torch.Tensor
    ent_j: torch.Tensor
    slot_u: torch.Tensor
    err: torch.Tensor
    bits: int
    nnz: int = 0
    gen: int = 0
    ecnt: torch.Tensor | None = None  # uint8 [tiles*TP_TILE] tail filter: entry occurrences
    cnt_pre: torch.Tensor | None = None  # tail filter: the counts before filtering
    flat = True

    @property
    def bufs(self):
        """(cnt, uniqf, ent_pos, ent_j, slot_u): the tuple the native ops take."""
        return (self.cnt, self.uniqf, self.ent_pos, self.ent_j, self.slot_u)

    def unique_keys(self) -> torch.Tensor:
        """Host sync: the distinct mixed keys in bucket order (key-range sorted across
        buckets, unsorted inside one) -- for tests and diagnostics."""
        H = hipops()
        g = H.tpf_groups(self.nnz, self.bits)
        kr = H.tpf_key_region()
        c = self.cnt[:4 * g].view(g, 4).cpu()
        u = self.uniqf[:g * kr].view(g, 2, kr // 2).cpu()
        parts = []
        for b in range(g):
            for s in range(2):
                parts.append(u[b, s, :int(c[b, 2 * s])])
        return torch.cat(parts)


def ensure_local_col(loc: "Localized") -> torch.Tensor:
    """local_col of a lazily localised "tp" minibatch (``Localizer(lazy_cols=True)``
    skips the per-occurrence gather: the fused forward/backward reads the tile entry
    map instead); runs the gather on first use."""
    t = getattr(loc, "tile", None)
    if t is not None and not t.cols_ready:
        hipops().tp_gather(t.rep, t.ent_uid, loc.nnz, loc.local_col)
        t.cols_ready = True
    return loc.local_col


class Localizer:
    """Reusable localisation workspace for up to ``max_nnz`` keys per call.

    ``mode="sort"``: radix sort + RLE (unique keys in sorted mixed order, CSC order
    for the segmented backward).
    ``mode="part"`` (csrc/hip/partloc.hip, GPU, key bits <= 32): one partition pass on
    the top key bits, then one workgroup per bucket deduplicates its keys in an LDS
    hash and sorts only the DISTINCT keys; same outputs as "sort" except the order of
    positions inside a key's segment (5 launches instead of 16).
    ``check()`` raises if a bucket overflowed its LDS hash (never for mixed keys of
    realistic batches; the bucket count bounds the distinct keys per bucket).
    ``mode="tp"`` (csrc/hip/tploc.hip, GPU, key bits <= 34, <= 5.2 M keys): LDS dedup of
    TP_TILE (8192)-occurrence tiles, then one workgroup per key-range bucket deduplicates the
    tile-distinct entries (a hot key is at most one entry per tile) and emits sorted
    unique keys, an entry-level CSC and local columns: 4 launches, no global atomics;
    the backward accumulates per tile in LDS and scans the entry CSC (``TileInfo``).
    ``mode="tpf"`` (1 GPU, same limits as "tp"): the tile stage of "tp", then bucket
    workgroups that write fixed per-bucket regions (``FlatLoc``): no look-back across
    buckets, no sort, no CSC; only the fused 1-GPU step consumes it (``tpf_step``). Its
    tiles hold 1024..8192 occurrences (``tpf_tile_log2``: >= ~128 tiles when the
    minibatch allows, so B = 10,000 fills the chip); tile entry ids keep the 8192 stride.
    (Measured and removed in round 3: a sort-free global scratch hash, a partition
    with per-bucket presence bitmaps and a 4096-key tile dedup + radix sort; none beat
    "tp" on the Criteo-shaped batch, profiles/r2_localize_tp_vs_sort.log.)"""

    def __init__(self, max_nnz: int, bits: int, device="cpu", with_hess: bool = False,
                 mode: str = "sort", lazy_cols: bool = False, sorted_keys: bool = False,
                 tail_filter=None):
        self.max_nnz = int(max_nnz)
        # "tpf": (CountMinSketch with key_bits = bits, freq) -> the fused tail filter of the
        # bucket kernel (tploc.hip tpf_filter_unit): filtered keys leave the minibatch
        self.tail_filter = tail_filter
        # "tpf": rank-sort each bucket's keys (the multi-GPU exchange rows stay key-ordered)
        self.sorted_keys = bool(sorted_keys)
        self.lazy_cols = bool(lazy_cols)  # "tp": local_col on demand (ensure_local_col)
        self.bits = int(bits)
        self.device = torch.device(device)
        self.with_hess = with_hess
        n = self.max_nnz
        dev = self.device
        self.gpu = dev.type == "cuda"
        self._tp_views = None  # (n, n-sized workspace views) of the last "tp" call
        if mode not in ("sort", "part", "tp", "tpf"):
            raise ValueError(f"unknown localisation mode {mode!r}")
        if mode == "part" and not (self.gpu and hipops().partloc_supported(n, self.bits)):
            mode = "sort"
        if mode in ("tp", "tpf") and (with_hess or not (self.gpu and
                                                        hipops().tploc_supported(n, self.bits))):
            mode = "sort"
        # (tp: up to 34-bit keys through its quotient-encoded tile hash)
        self.mode = mode if (self.gpu and (self.bits <= 32 or mode in ("tp", "tpf"))) else "sort"
        if self.gpu and self.mode == "tpf":
            H = hipops()
            # (smaller minibatches may use more, smaller tiles: the bound over n' <= n)
            N = H.tpf_stride_max(n)
            g = H.tpf_groups(n, self.bits)  # the largest geometry (fewer keys: fewer groups)
            kr, er = H.tpf_key_region(), H.tpf_entry_region()
            self.ptemp = torch.empty(H.tpf_temp_bytes(n, self.bits), dtype=torch.uint8, device=dev)
            i32 = lambda k: torch.zeros(k, dtype=torch.int32, device=dev)  # noqa: E731
            self.flat = FlatLoc(
                rep=torch.empty(n, dtype=torch.int16, device=dev), dcnt=i32(N // TP_TILE),
                psum=torch.zeros(N, dtype=torch.float32, device=dev),
                w_ent=torch.zeros(N, dtype=torch.float32, device=dev),
                cnt=i32(4 * g), uniqf=torch.zeros(g * kr, dtype=torch.int64, device=dev),
                ent_pos=i32(g * er), ent_j=torch.zeros(g * er, dtype=torch.int16, device=dev),
                slot_u=i32(g * kr), err=i32(1), bits=self.bits,
                ecnt=(torch.zeros(N, dtype=torch.uint8, device=dev) if tail_filter is not None
                      else None),
                cnt_pre=i32(4 * g) if tail_filter is not None else None)
            self.err = self.flat.err
            return
        if self.gpu and self.mode == "tp":
            H = hipops()
            N = H.tploc_stride(n)
            i32 = lambda k: torch.empty(k, dtype=torch.int32, device=dev)  # noqa: E731
            # zeroed once: the bucket look-back's status words + launch epoch (tploc.hip)
            self.ptemp = torch.zeros(H.tploc_temp_bytes(n, self.bits), dtype=torch.uint8,
                                     device=dev)
            self.t_dcnt, self.t_rep = i32(N // TP_TILE), torch.empty(n, dtype=torch.int16, device=dev)
            self.pos_s, self.segid, self.t_ent_uid = i32(N), i32(N), i32(N)
            self.seg_start, self.local_col = i32(N + 1), i32(n)
            self.uniq = torch.empty(N, dtype=torch.int64, device=dev)
            self.n_uniq = torch.zeros(1, dtype=torch.int32, device=dev)
            self.t_nent = torch.zeros(1, dtype=torch.int32, device=dev)
            self.grad = torch.empty(N, dtype=torch.float32, device=dev)
            self.t_psum = torch.empty(N, dtype=torch.float32, device=dev)
            self.t_pieces = torch.empty(N, dtype=torch.int64, device=dev)
            self.hess = None
            self.err = torch.zeros(1, dtype=torch.int32, device=dev)
            return
        if self.gpu and self.mode == "part":
            H = hipops()
            i32 = lambda k: torch.empty(k, dtype=torch.int32, device=dev)  # noqa: E731
            self.ptemp = torch.empty(H.partloc_temp_bytes(n, self.bits), dtype=torch.uint8,
                                     device=dev)
            self.pos_s, self.segid, self.local_col = i32(n), i32(n), i32(n)
            self.seg_start = i32(n + 1)
            self.uniq = torch.empty(n, dtype=torch.int64, device=dev)
            self.n_uniq = torch.zeros(1, dtype=torch.int32, device=dev)
            self.grad = torch.empty(n, dtype=torch.float32, device=dev)
            self.hess = torch.empty(n, dtype=torch.float32, device=dev) if with_hess else None
            self.err = torch.zeros(1, dtype=torch.int32, device=dev)
            return
        if self.gpu:
            H = hipops()
            self.h = torch.empty(n, dtype=torch.int64, device=dev)
            self.hs = torch.empty(n, dtype=torch.int64, device=dev)
            self.pos = torch.empty(n, dtype=torch.int32, device=dev)
            self.pos_s = torch.empty(n, dtype=torch.int32, device=dev)
            self.flags = torch.empty(n, dtype=torch.int32, device=dev)
            self.segid = torch.empty(n, dtype=torch.int32, device=dev)
            self.uniq = torch.empty(n, dtype=torch.int64, device=dev)
            self.seg_start = torch.empty(n + 1, dtype=torch.int32, device=dev)
            self.local_col = torch.empty(n, dtype=torch.int32, device=dev)
            self.n_uniq = torch.zeros(1, dtype=torch.int32, device=dev)
            self.grad = torch.empty(n, dtype=torch.float32, device=dev)
            self.hess = torch.empty(n, dtype=torch.float32, device=dev) if with_hess else None
            self.fast32 = self.bits <= 32
            # digit width of the u32 radix sort: 10-bit digits sort 21..30-bit keys in 3
            # passes (vs 4 with 8 bits); PSAMD_SORT_DIGIT_BITS overrides for A/B runs
            import os

            db = int(os.environ.get("PSAMD_SORT_DIGIT_BITS", "0"))
            self.digit_bits = db if db in (8, 10) else (10 if 24 < self.bits <= 30 else 8)
            if self.fast32:  # fused mix + u32 radix sort + fused RLE (csrc/hip/sort32.hip)
                self.hs32 = torch.empty(n, dtype=torch.int32, device=dev)
                self.sort_temp = torch.empty(H.localize32_temp_bytes(n), dtype=torch.uint8,
                                             device=dev)
            else:
                self.sort_temp = torch.empty(max(1, H.sort_pairs_temp_bytes(n, self.bits)),
                                             dtype=torch.uint8, device=dev)
            # 33..40-bit keys (10^10 features), < 2^22 keys: 4 x 10-bit u32 passes with the
            # high key bits carried next to the position (sort32.hip sort40) instead of
            # the generic 5 x 8-bit u64 sort (65,536 x 39 keys at 34 bits: 420 -> 257 us)
            self.fast40 = 32 < self.bits <= 40 and n < (1 << 22) and \
                os.environ.get("PSAMD_SORT40", "1") != "0"
            if self.fast40:
                self.sort40_temp = torch.empty(H.sort40_temp_bytes(n), dtype=torch.uint8,
                                               device=dev)
            self.scan_temp = torch.empty(max(1, H.scan_temp_bytes(n)), dtype=torch.uint8,
                                         device=dev)

    def filt_args(self):
        """The native fused tail filter's argument tuple ("tpf" with a tail filter) or None."""
        if self.tail_filter is None or self.mode != "tpf":
            return None
        cm, freq = self.tail_filter
        if cm.rshift >= 64 or cm.key_bits != self.bits:
            raise ValueError("the fused tail filter needs a CountMinSketch partitioned over "
                             "this localiser's key bits")
        return (*cm.args(freq), self.flat.ecnt, self.flat.w_ent, self.flat.cnt_pre)

    def check(self):
        """Host sync: raise if a "part" localisation overflowed a bucket's LDS hash."""
        if getattr(self, "err", None) is not None and self.mode in ("part", "tp", "tpf") and \
                int(self.err.item()):
            raise RuntimeError(f"localize_{self.mode}: a bucket or tile overflowed its LDS capacity")

    def __call__(self, keys: torch.Tensor, stage: int = 0) -> Localized:
        """``stage`` (flat layout with a tail filter): 4 = tile + bucket kernels, 3 = the
        filter kernel (a caller orders the filters of consecutive minibatches between
        the two calls); 0 = all."""
        n = keys.numel()
        if n > self.max_nnz:
            raise ValueError(f"minibatch has {n} keys > workspace {self.max_nnz}")
        if n == 0:
            raise ValueError("empty minibatch")
        if stage and (self.mode != "tpf" or self.tail_filter is None or stage not in (3, 4)):
            raise ValueError("staged localisation: the flat layout with a tail filter, 4 / 3")
        if self.gpu and is_gpu(keys):
            return self._gpu(keys.contiguous(), n, stage)
        if self.mode == "tpf":
            raise ValueError("a flat (tpf) localiser takes GPU keys")
        return localize_torch(keys, self.bits, self.with_hess)

    def _gpu(self, keys, n, stage=0) -> Localized:
        H = hipops()
        if self.mode == "tpf":
            f = self.flat
            H.localize_tpf(keys, self.bits, self.ptemp, f.dcnt, f.rep, f.uniqf, f.ent_pos,
                           f.ent_j, f.cnt, f.err, self.sorted_keys, filt=self.filt_args(),
                           stage=stage)
            if stage != 4:  # (a new generation once the minibatch is complete)
                f.nnz = n
                f.gen += 1
            return f
        if self.mode == "tp":
            # the look-back's status words carry an 8-bit launch epoch: when the bucket
            # count changes (another minibatch size), a bucket left unused for exactly
            # 255 launches could accept a stale word -> zero them (and the epoch) then
            nbk = H.tploc_buckets(n, self.bits)
            if nbk != getattr(self, "_last_nbk", None):
                if getattr(self, "_last_nbk", None) is not None:
                    self.ptemp[:(max(nbk, self._last_nbk) * 8 + 16 + 15) // 16 * 16].zero_()
                self._last_nbk = nbk
            H.localize_tp(keys, self.bits, self.ptemp, self.t_dcnt, self.t_rep, self.pos_s,
                          self.segid, self.uniq, self.seg_start, self.t_ent_uid,
                          None if self.lazy_cols else self.local_col,
                          self.n_uniq, self.t_nent, self.grad, self.t_pieces, self.err,
                          getattr(self, "tp_prof", None))
            # unique keys <= n: expose n-sized views (the workspace is tile-rounded); the
            # views of the last n are kept (4 slices are ~4 us of host time per call)
            v = self._tp_views
            if v is None or v[0] != n:
                v = self._tp_views = (n, self.uniq[:n], self.local_col[:n], self.grad[:n],
                                      self.t_pieces[:n])
            tile = TileInfo(self.t_rep, self.t_dcnt, self.t_nent, self.t_psum, self.t_ent_uid,
                            not self.lazy_cols, v[4])
            return Localized(v[1], self.seg_start, self.pos_s, self.segid, v[2], self.n_uniq,
                             v[3], None, n, tile=tile)
        if self.mode == "part":
            H.localize_part(keys, self.bits, self.ptemp, self.pos_s, self.segid, self.uniq,
                            self.seg_start, self.local_col, self.n_uniq, self.grad, self.hess,
                            self.err)
            return Localized(self.uniq, self.seg_start, self.pos_s[:n], self.segid[:n],
                             self.local_col[:n], self.n_uniq, self.grad, self.hess, n)
        if self.fast32:
            H.localize32(keys, self.bits, self.sort_temp, self.hs32, self.pos_s, self.segid,
                         self.uniq, self.seg_start, self.local_col, self.n_uniq, self.grad,
                         self.hess, self.digit_bits)
            return Localized(self.uniq, self.seg_start, self.pos_s[:n], self.segid[:n],
                             self.local_col[:n], self.n_uniq, self.grad, self.hess, n)
        if self.fast40:
            H.sort40(keys, self.bits, self.sort40_temp, self.hs, self.pos_s)
        else:
            H.mix_iota(keys, self.bits, self.h, self.pos)
            H.sort_pairs(self.sort_temp, self.h, self.hs, self.pos, self.pos_s, n, self.bits)
        H.rle(self.hs, self.pos_s, n, self.flags, self.segid, self.scan_temp, self.uniq,
              self.seg_start, self.local_col, self.n_uniq, self.grad, self.hess)
        return Localized(self.uniq, self.seg_start, self.pos_s[:n], self.segid[:n],
                         self.local_col[:n], self.n_uniq, self.grad, self.hess, n)


def localize_torch(keys: torch.Tensor, bits: int, with_hess: bool = False) -> Localized:
    """Plain-PyTorch localisation (CPU path and numerics reference)."""
    h = mix(keys.contiguous(), bits)
    order_key = to_unsigned_order(h) if bits == 64 else h
    sk, perm = torch.sort(order_key, stable=True)
    hs = h[perm]
    uniq, counts = torch.unique_consecutive(hs, return_counts=True)
    U = uniq.numel()
    seg = torch.repeat_interleave(torch.arange(U, device=keys.device), counts)
    local_col = torch.empty(keys.numel(), dtype=torch.int32, device=keys.device)
    local_col[perm] = seg.to(torch.int32)
    seg_start = torch.zeros(U + 1, dtype=torch.int32, device=keys.device)
    seg_start[1:] = torch.cumsum(counts, 0).to(torch.int32)
    return Localized(uniq, seg_start, perm.to(torch.int32), (seg + 1).to(torch.int32), local_col,
                     torch.tensor([U], dtype=torch.int32, device=keys.device),
                     torch.zeros(U, dtype=torch.float32, device=keys.device),
                     torch.zeros(U, dtype=torch.float32, device=keys.device) if with_hess else None,
                     keys.numel())
