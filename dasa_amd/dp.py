"""Episode-sharded data parallelism for Seq2SeqAgent.

One process per GPU; each rank runs its own environment/episode stream. Replicas start identical
(rank-0 broadcast) and stay identical because the only exchange — one all-reduce (sum / world) of a
flat fp32 bucket holding every gradient the step produced — happens before clip_grad_norm and
RMSprop (agent_dg.py:1389-1405), which then run the same math on every rank. Backend "nccl" is
RCCL on ROCm (xGMI inside a node). Parameters without a gradient anywhere (the detached BERT stack,
unused linear_out heads) are excluded, and a parameter keeps `grad=None` iff no rank produced one,
so the optimizer skips exactly what the single-GPU reference skips.
"""
import torch
import torch.distributed as dist


class GradSync:
    """One flat-bucket all-reduce of the gradient-receiving parameters per optimizer step.

    Which parameters received a gradient on ANY rank is agreed every step (a small mask all-reduce), so a
    mode switch (e.g. teacher-only iterations, where the critic gets none) stays exact. The mask
    all-reduce is enqueued by `prepare()` before optim_step's device-error-word read, and its host read
    in `__call__` comes after it: the step's one host sync (the error-word check, which must precede
    clipping and the optimizers anyway) covers both — no second sync per step. The host-side local mask
    is cached per gradient set, so no host->device copy is made either."""

    def __init__(self, params, bucket_mb=256):
        self.params = [p for p in params if p.requires_grad]
        self.world = dist.get_world_size()
        self.numel = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.empty(self.numel, dtype=torch.float32, device=dev)
        self.mask = torch.empty(len(self.params), dtype=torch.float32, device=dev)
        self.bucket = max(1, int(bucket_mb * 2**20 / 4))
        self.sent = 0            # floats all-reduced by the last call
        self._local = {}         # gradient set (tuple of bools) -> its mask on the device
        self._prepared = False

    def prepare(self):
        """Enqueue the mask all-reduce (no host sync). Call after backward, before the host sync that
        precedes __call__; __call__ does it itself when it was not called."""
        local = tuple(p.grad is not None for p in self.params)
        m = self._local.get(local)
        if m is None:
            m = self._local[local] = self.mask.new_tensor([1.0 if g else 0.0 for g in local])
        self.mask.copy_(m)
        dist.all_reduce(self.mask)
        self._prepared = True

    def __call__(self):
        # which parameters received a gradient on ANY rank: only those travel in the bucket — the
        # 47.23 M floats of the README train config, not the 58 M trainable ones (the unused linear_out
        # heads, encoder2decoder_*, never get one)
        if not self._prepared:
            self.prepare()
        self._prepared = False
        m = self.mask.cpu().tolist()
        off = 0
        for p, any_rank in zip(self.params, m):
            if any_rank > 0:
                n = p.numel()
                if p.grad is not None:
                    self.flat[off:off + n].copy_(p.grad.view(-1))
                else:
                    self.flat[off:off + n].zero_()
                off += n
        self.sent = off
        # bucketed so that very large models keep several collectives in flight on RCCL's channels
        for s in range(0, off, self.bucket):
            dist.all_reduce(self.flat[s:min(off, s + self.bucket)])
        self.flat[:off].div_(self.world)
        off = 0
        for p, any_rank in zip(self.params, m):
            if any_rank > 0:
                n = p.numel()
                g = self.flat[off:off + n].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
                off += n


def broadcast_params(modules, src=0):
    for m in modules:
        for t in list(m.parameters()) + list(m.buffers()):
            dist.broadcast(t.data, src)


def _trainable(agent):
    """Parameters that can receive gradients in this configuration."""
    out = []
    for m in agent.models:
        for name, p in m.named_parameters():
            if m is agent.encoder and name.startswith("bert."):
                bert = agent.encoder.bert
                lang = name.startswith("bert.embeddings") or name.startswith("bert.lalayer") or \
                    name.startswith("bert.pooler")
                if lang and not bert.update_lang_bert:
                    continue
                if not lang and not bert.update_add_layer:
                    continue
            out.append(p)
    return out


def attach(agent, force=False):
    """Broadcast rank 0's weights and install the gradient all-reduce in agent.optim_step().
    `force` (test hook) installs it at world size 1 too, so the collective path runs on one GPU.

    Every rank of an unchanged train.py seeds torch identically (train.py:521), so the random streams
    are made rank-specific here: torch's generator (nn.Dropout, the env-drop noise) is re-seeded with
    seed + 7919 * rank, and the counter-RNG seed stream of the HIP kernels (dropout masks, Categorical
    draws) gets the rank as salt. Rank 0 keeps the single-GPU streams."""
    if not dist.is_initialized() or (dist.get_world_size() == 1 and not force):
        return None
    from . import functional as DF
    rank = dist.get_rank()
    if rank:
        torch.manual_seed((torch.initial_seed() + 7919 * rank) % (2**63))
    DF.set_rank_salt(rank)
    broadcast_params(agent.models)
    sync = GradSync(_trainable(agent))
    agent.grad_sync = sync
    return sync
