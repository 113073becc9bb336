"""Owner-side push apply of all G source rows in one launch: the key-range
partitioned kernel (kv_apply_part) against the chained-hash pair (kv_update_rows,
itself checked against per-row sequential launches in test_dist_gpu). Bitwise
equal slot tables: the same per-key update sequence in source-rank order.
Reference semantics: every push is its own optimizer step (src/parameter/kv_store.h:47-57)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rows(G, C, n_per, span, lo, seed, nan_frac=0.0, dup_pool=None):
    """Exchange rows [nkeys, ngrads, -, -, keys (u32), grads]: row s holds n_per[s] sorted
    distinct keys in [lo, lo + span), many shared across rows."""
    g = torch.Generator().manual_seed(seed)
    H = (4 + C + C + 3) // 4 * 4
    recv = torch.zeros(G * H, dtype=torch.int32)
    pool = dup_pool if dup_pool is not None else torch.randperm(span, generator=g)[: 3 * max(n_per)]
    for s in range(G):
        n = n_per[s]
        pick = pool[torch.randperm(pool.numel(), generator=g)[:n]]
        keys = torch.sort(pick + lo).values
        grads = torch.randn(n, generator=g)
        if nan_frac:
            grads[torch.rand(n, generator=g) < nan_frac] = float("nan")
        row = recv[s * H:(s + 1) * H]
        row[0] = n
        row[1] = n
        row[4:4 + n] = keys.to(torch.int64).to(torch.int32)  # u32 bit pattern
        row[4 + C:4 + C + n] = grads.view(torch.int32)
    return recv, H


@pytest.mark.parametrize("G,C,lgP,nan", [(1, 256, 2, 0.0), (3, 2048, 3, 0.0), (8, 4096, 6, 0.1),
                                         (8, 4096, 0, 0.0), (5, 1024, 9, 0.05)])
def test_partitioned_apply_matches_chained(G, C, lgP, nan):
    from parameter_server_amd.ops.native import hipops
    from parameter_server_amd.ops.kv_table import KVTable, UpdateRule, next_pow2

    dev = torch.device("cuda")
    lo, span = 1 << 20, 1 << 22
    n_per = [C - 7 * s for s in range(G)]
    recv, H = _rows(G, C, n_per, span, lo, seed=G * 100 + lgP, nan_frac=nan)
    recv = recv.to(dev)
    tabs = [KVTable(1 << 16, dev, key_range=(lo, lo + span)) for _ in range(2)]
    rule = UpdateRule(algo="ftrl", alpha=0.1, beta=1.0, l1=0.5, l2=0.1)
    hh = hipops()
    P = 1 << lgP
    slot = torch.full((G * C,), -1, dtype=torch.int64, device=dev)
    w = torch.zeros(G * C, dtype=torch.float32, device=dev)
    keys = torch.zeros(G * C, dtype=torch.int64, device=dev)
    bnd = torch.full((G * (P + 1),), -5, dtype=torch.int32, device=dev)
    tb = tabs[0]
    it, iv, isd, seed = tb.init.args()
    hh.kv_resolve_rows(tb.slots, recv, H, C, 1, slot, w, True, it, iv, isd, seed, tb._err,
                       None, tb.home_base, tb.home_m, keys, bnd, lgP)
    tabs[1].slots.copy_(tb.slots)  # same placement (insert races may differ per table)
    torch.cuda.synchronize()
    # bounds: row s, partition q -> number of its keys with part(key) < q
    b = bnd.view(G, P + 1).cpu()
    assert (b[:, 0] == 0).all() and (b[:, P] == torch.tensor(n_per)).all()
    assert (b[:, 1:] >= b[:, :-1]).all()
    k_host = keys.view(G, C).cpu()
    for s in range(G):
        assert torch.equal(k_host[s, :n_per[s]] & 0xFFFFFFFF,
                           recv.view(G, H)[s, 4:4 + n_per[s]].cpu().to(torch.int64) & 0xFFFFFFFF)
    # a second push round on top of the first exercises non-zero optimizer state
    for _ in range(2):
        gsrc = recv.view(torch.float32)[4 + C:]
        st = [torch.zeros(3, dtype=torch.float64, device=dev) for _ in range(2)]
        link = torch.empty(next_pow2(2 * G * C), dtype=torch.int64, device=dev)
        nxt = torch.empty(G * C, dtype=torch.int32, device=dev)
        hh.kv_update_rows(tabs[0].slots, slot, gsrc, H, recv, H, C, link, nxt, *rule.args(), st[0])
        hh.kv_apply_part(tabs[1].slots, slot, keys, gsrc, H, recv, H, C, bnd, lgP, *rule.args(),
                         st[1])
        torch.cuda.synchronize()
        assert torch.equal(tabs[0].slots, tabs[1].slots)
        torch.testing.assert_close(st[0], st[1], rtol=1e-9, atol=1e-9)
    assert (tabs[1].slots.view(torch.int32)[:, 2].view(torch.float32) != 0).any()  # w moved


def test_partitioned_apply_many_windows():
    """Every key in one partition (lgP = 0) with rows far longer than the 1024-entry
    LDS window: the window loop must keep each key's entries together."""
    from parameter_server_amd.ops.native import hipops
    from parameter_server_amd.ops.kv_table import KVTable, UpdateRule, next_pow2

    dev = torch.device("cuda")
    G, C, lo, span = 6, 8192, 0, 1 << 16
    pool = torch.randperm(span, generator=torch.Generator().manual_seed(3))[:9000]
    recv, H = _rows(G, C, [C - 100 * s for s in range(G)], span, lo, seed=5, dup_pool=pool)
    recv = recv.to(dev)
    rule = UpdateRule(algo="sgd", alpha=0.05)
    tabs = [KVTable(1 << 15, dev, key_range=(lo, lo + span)) for _ in range(2)]
    hh = hipops()
    slot = torch.full((G * C,), -1, dtype=torch.int64, device=dev)
    w = torch.zeros(G * C, dtype=torch.float32, device=dev)
    keys = torch.zeros(G * C, dtype=torch.int64, device=dev)
    bnd = torch.zeros(G * 2, dtype=torch.int32, device=dev)
    tb = tabs[0]
    it, iv, isd, seed = tb.init.args()
    hh.kv_resolve_rows(tb.slots, recv, H, C, 1, slot, w, True, it, iv, isd, seed, tb._err,
                       None, tb.home_base, tb.home_m, keys, bnd, 0)
    tabs[1].slots.copy_(tb.slots)
    gsrc = recv.view(torch.float32)[4 + C:]
    link = torch.empty(next_pow2(2 * G * C), dtype=torch.int64, device=dev)
    nxt = torch.empty(G * C, dtype=torch.int32, device=dev)
    hh.kv_update_rows(tabs[0].slots, slot, gsrc, H, recv, H, C, link, nxt, *rule.args(), None)
    hh.kv_apply_part(tabs[1].slots, slot, keys, gsrc, H, recv, H, C, bnd, 0, *rule.args(), None)
    torch.cuda.synchronize()
    assert torch.equal(tabs[0].slots, tabs[1].slots)


@pytest.mark.parametrize("G,C,lgP,post", [(2, 4096, 5, True), (8, 2048, 9, True),
                                          (8, 2048, 9, False), (3, 1024, 0, True)])
def test_owner_part_matches_resolve_then_apply(G, C, lgP, post):
    """kv_owner_part (one launch: resolve of the pulled keys with the SENDER's partition
    bounds from xchg_pack_keys, then the per-source apply of an earlier pull) leaves the
    table, slots, weights and bounds of kv_resolve_rows + kv_apply_part run separately
    (post = resolve first; pre = apply first)."""
    from parameter_server_amd.ops.kv_table import KVTable, UpdateRule
    from parameter_server_amd.ops.native import hipops

    dev = torch.device("cuda")
    H = hipops()
    P = 1 << lgP
    kw = 2
    gw = C
    w0 = 4 + C * kw + gw
    b0 = w0 + C
    Hr = (b0 + P + 1 + 3) // 4 * 4
    lo, hi = 1 << 40, 1 << 44
    rule = UpdateRule("ftrl", "decay", 0.05, 1.0, 0.1, 0.1)
    g = torch.Generator(device=dev).manual_seed(7)

    def table():
        return KVTable(1 << 16, dev, key_range=(lo, hi))

    def sorted_keys(n):
        return torch.unique(torch.randint(lo, hi, (n,), device=dev, generator=g))

    # an earlier pull (the push's slots / keys / bounds) and this exchange's pulls
    old_keys = [sorted_keys(int(C * 0.6)) for _ in range(G)]
    new_keys = [torch.cat([old_keys[s][::3], sorted_keys(C // 3)]).unique()[:C - 8]
                for s in range(G)]
    gr = torch.randn(G * C, device=dev, generator=g)  # (the same pushes in both runs)
    outs = []
    for fused in (True, False):
        tb = table()
        homes = torch.tensor([[tb.home_base - (1 << 64) if tb.home_base >= 1 << 63 else
                               tb.home_base, tb.home_m - (1 << 64) if tb.home_m >= 1 << 63
                               else tb.home_m]] * G, dtype=torch.int64, device=dev)
        it, iv, isd, seed = tb.init.args()
        # earlier pull: resolve old keys -> slots_old / keys_old / bnd_old
        recv_old = torch.zeros(G * Hr, dtype=torch.int32, device=dev)
        ukeys = torch.cat(old_keys)
        off = torch.tensor([0] + torch.cumsum(torch.tensor([k.numel() for k in old_keys]), 0)
                           .tolist(), dtype=torch.int64, device=dev)
        n_u = torch.tensor([ukeys.numel()], dtype=torch.int32, device=dev)
        # (the rows of one sender to G owners = one exchange's received rows here)
        H.xchg_pack_keys(ukeys, n_u, off, C, kw, Hr, recv_old, None, homes=homes, b0=b0, lgP=lgP)
        slots_old = torch.full((G * C,), -1, dtype=torch.int64, device=dev)
        keys_old = torch.zeros(G * C, dtype=torch.int64, device=dev)
        bnd_old = torch.zeros(G * (P + 1), dtype=torch.int32, device=dev)
        wtmp = torch.zeros(G * C, dtype=torch.float32, device=dev)
        H.kv_resolve_rows(tb.slots, recv_old, Hr, C, kw, slots_old, wtmp, True, it, iv, isd, seed,
                          tb._err, None, tb.home_base, tb.home_m, keys_old, bnd_old, lgP)
        # the rows' sender bounds equal the resolve's bounds
        rb = torch.stack([recv_old[s * Hr + b0:s * Hr + b0 + P + 1] for s in range(G)])
        assert torch.equal(rb.reshape(-1), bnd_old)
        # this exchange: new keys + gradients of the old pull
        recv = torch.zeros(G * Hr, dtype=torch.int32, device=dev)
        ukeys = torch.cat(new_keys)
        off = torch.tensor([0] + torch.cumsum(torch.tensor([k.numel() for k in new_keys]), 0)
                           .tolist(), dtype=torch.int64, device=dev)
        n_u = torch.tensor([ukeys.numel()], dtype=torch.int32, device=dev)
        H.xchg_pack_keys(ukeys, n_u, off, C, kw, Hr, recv, None, homes=homes, b0=b0, lgP=lgP)
        for s in range(G):
            n = old_keys[s].numel()
            recv[s * Hr + 1] = n
            recv[s * Hr + 4 + C * kw:s * Hr + 4 + C * kw + n] = gr[s * C:s * C + n].view(torch.int32)
        gsrc = recv.view(torch.float32)[4 + C * kw:]
        slots_new = torch.full((G * C,), -1, dtype=torch.int64, device=dev)
        keys_new = torch.zeros(G * C, dtype=torch.int64, device=dev)
        bnd_new = torch.zeros(G * (P + 1), dtype=torch.int32, device=dev)
        sendn = torch.zeros(G * Hr, dtype=torch.int32, device=dev)
        wout = sendn.view(torch.float32)[w0:]
        from parameter_server_amd.ops.linear import new_accum

        stats = new_accum(dev)
        if fused:
            H.kv_owner_part(tb.slots, recv, Hr, C, kw, b0, lgP, slots_new, keys_new, bnd_new, wout,
                            it, iv, isd, seed, tb._err, None, tb.home_base, tb.home_m, slots_old,
                            keys_old, gsrc, Hr, bnd_old, post, *rule.args(), stats)
        else:
            def res():
                H.kv_resolve_rows(tb.slots, recv, Hr, C, kw, slots_new, wout, True, it, iv, isd,
                                  seed, tb._err, None, tb.home_base, tb.home_m, keys_new, bnd_new,
                                  lgP, wstride=Hr)

            def app():
                H.kv_apply_part(tb.slots, slots_old, keys_old, gsrc, Hr, recv, Hr, C, bnd_old,
                                lgP, *rule.args(), stats)
            (res(), app()) if post else (app(), res())
        torch.cuda.synchronize()
        k, w, z, n = tb.occupied()
        o = torch.argsort(k)
        W = torch.stack([wout[s * Hr:s * Hr + new_keys[s].numel()] for s in range(G)], 0) \
            if len({k_.numel() for k_ in new_keys}) == 1 else torch.cat(
                [wout[s * Hr:s * Hr + new_keys[s].numel()] for s in range(G)])
        outs.append((k[o].cpu(), w[o].cpu(), z[o].cpu(), n[o].cpu(), W.cpu(), bnd_new.cpu(),
                     keys_new.cpu()))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    assert int(tb._err.item()) == 0
