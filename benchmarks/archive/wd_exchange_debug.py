import os, sys, socket
sys.path.insert(0, os.getcwd())
import torch, numpy as np
import torch.multiprocessing as mp

def worker(rank, world, port, q, exchange, steps):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parameter_server_amd.models.wide_deep import WideDeepConfig, WideDeepTrainer
    from parameter_server_amd.ops.synthetic import criteo_batch
    from parameter_server_amd.parallel.comm import DistComm
    from parameter_server_amd.ops.kv_table import EMPTY_KEY
    dev = torch.device("cuda", 0)
    comm = DistComm(dev)
    cfg = WideDeepConfig(num_features=1 << 22, embedding_dim=64, hidden=(256, 128), minibatch=1024,
                         table_capacity=1 << 16, exchange=exchange)
    tr = WideDeepTrainer(cfg, comm, dev)
    for s in range(steps):
        k, l = criteo_batch(1024, seed=50 + rank, row0=s * 1024, num_features=1 << 22, cards=[1000] * 26, device=dev)
        tr.step(k, l)
    torch.cuda.synchronize()
    idx = torch.nonzero(tr.shard.table.slots[:, 0] != EMPTY_KEY).flatten()
    keys, w, _, _ = tr.shard.table.occupied()
    o = torch.argsort(keys)
    rows = tr.shard.rows[idx[o]].float().cpu()
    q.put((rank, keys[o].cpu().numpy(), rows.numpy(), tr.param.cpu().numpy()))
    dist.barrier(); dist.destroy_process_group()

def run(exchange, steps):
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn"); q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, 2, port, q, exchange, steps)) for r in range(2)]
    for p in ps: p.start()
    res = sorted([q.get(timeout=120) for _ in ps], key=lambda r: r[0])
    for p in ps: p.join(60)
    return res

if __name__ == "__main__":
    for steps in (1, 2, 6):
        a, b = run("padded", steps), run("exact", steps)
        for ra, rb in zip(a, b):
            assert (ra[1] == rb[1]).all()
            d = np.abs(ra[2] - rb[2]).max(axis=1)
            bad = np.nonzero(d > 1e-3)[0]
            print(f"steps {steps} rank {ra[0]}: keys {len(d)} rows differing {len(bad)} max {d.max():.4g} param max diff {np.abs(ra[3]-rb[3]).max():.3g}", flush=True)
