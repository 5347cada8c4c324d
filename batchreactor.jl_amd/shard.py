"""Ensemble sharding across GPUs: one process per GPU, reactors independent.

Strong scaling (the BASELINE.json configs: a fixed ensemble of N_total reactors sharded over
1/2/4/8 GPUs): rank r of W integrates the contiguous slice shard_range(r, W, N_total) (sizes differ
by at most one). Weak scaling: rank r integrates [r*N, (r+1)*N). Inputs are generated per rank
from the counter-based splitmix64 stream, so no input is communicated. The integration itself has
no collective; after it, one all-gather returns the final states and solver counters to every
rank in ensemble order, and the step time is the maximum over ranks. Within a GPU the persistent
kernel's work counter balances the stiffness variance between reactors. Backend "nccl" (RCCL over
xGMI) on the GPU box, "gloo" in the CPU tests -- the code path is the same.
"""


def shard_slice(rank: int, per_rank: int):
    """[start, stop) of this rank's reactors (weak scaling: per_rank reactors per rank)."""
    return rank * per_rank, (rank + 1) * per_rank


def shard_range(rank: int, world: int, total: int):
    """[start, stop) of this rank's reactors when `total` reactors are split over `world` ranks
    (strong scaling): contiguous, in ensemble order, the first total % world ranks one longer."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """The slowest rank's time (the bench contract: max over ranks)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_ensemble(U, stats, dist=None, total=None):
    """All-gather this rank's final states U[N_r, n] and stats[N_r, k] (torch tensors on the rank's
    device: HIP for nccl, CPU for gloo) into [sum N_r, n] / [sum N_r, k] in ensemble order. With
    `total` (strong scaling) the slices may differ in length by one: they are padded to the
    longest for the collective and trimmed after it."""
    import torch
    payload = torch.cat([U, stats], dim=1).contiguous()
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        out = payload
    else:
        world = dist.get_world_size()
        sizes = [shard_range(r, world, total)[1] - shard_range(r, world, total)[0] for r in range(world)] \
            if total is not None else [payload.shape[0]] * world
        m = max(sizes)
        if payload.shape[0] < m:
            payload = torch.cat([payload, payload.new_zeros((m - payload.shape[0], payload.shape[1]))], dim=0)
        parts = [torch.empty_like(payload) for _ in range(world)]
        dist.all_gather(parts, payload)
        out = torch.cat([p[:s] for p, s in zip(parts, sizes)], dim=0)
    n = U.shape[1]
    return out[:, :n], out[:, n:]
