"""Data-parallel gradient exchange (dasa_amd.dp) with world_size 2 over gloo on the CPU: the same
code path the MI355X ranks run over RCCL (backend "nccl")."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dasa_amd.dp import GradSync, broadcast_params
    torch.manual_seed(100 + rank)            # replicas start different ...
    m = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Linear(5, 3), torch.nn.Linear(3, 2))
    broadcast_params([m])                    # ... until rank 0's weights are broadcast
    sync = GradSync(list(m.parameters()), bucket_mb=1e-5)   # tiny buckets: exercises the bucket loop
    x = torch.randn(4, 6) * (rank + 1)
    y = m(x)
    loss = y[:, 0].sum() if rank == 0 else y.sum()
    loss.backward()
    m[2].bias.grad = None if rank == 1 else m[2].bias.grad     # a grad present on one rank only
    m[0].weight.grad = None                                   # ... and a grad present on no rank
    local = {k: (p.grad.clone() if p.grad is not None else None) for k, p in m.named_parameters()}
    sync.prepare()                           # mask all-reduce enqueued ahead of the step's host sync
    sync()
    out = {k: (p.grad.clone() if p.grad is not None else None) for k, p in m.named_parameters()}
    weights = {k: p.detach().clone() for k, p in m.named_parameters()}
    # by value (numpy): shared-memory tensors would need this process alive until the parent reads them
    npd = lambda d: {k: (v.numpy() if v is not None else None) for k, v in d.items()}  # noqa: E731
    q.put((rank, npd(local), npd(out), npd(weights)))
    dist.barrier()
    dist.destroy_process_group()


def test_grad_allreduce_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, local, out, w = q.get(timeout=120)
        tt = lambda d: {k: (torch.from_numpy(v) if v is not None else None) for k, v in d.items()}  # noqa: E731
        res[r] = (tt(local), tt(out), tt(w))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (l0, o0, w0), (l1, o1, w1) = res[0], res[1]
    for k in w0:
        assert torch.equal(w0[k], w1[k]), "replicas must start identical after the broadcast"
    for k in o0:
        if l0[k] is None and l1[k] is None:
            assert o0[k] is None and o1[k] is None, k            # no rank produced it: stays None
            continue
        g0 = l0[k] if l0[k] is not None else torch.zeros_like(l1[k])
        g1 = l1[k] if l1[k] is not None else torch.zeros_like(l0[k])
        exp = (g0 + g1) / 2
        assert torch.allclose(o0[k], exp, atol=1e-6) and torch.allclose(o1[k], exp, atol=1e-6), k
