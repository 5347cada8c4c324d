"""Ensemble sharding across GPUs: one process per GPU, reactors independent.

Rank r of W integrates the contiguous slice [r*N, (r+1)*N) of the ensemble (weak scaling: N
reactors per GPU, inputs generated per rank from the counter-based splitmix64 stream, so no
input is communicated). The integration itself has no collective; after it, one all-gather
returns the final states and solver counters to every rank in ensemble order, and the step time
is the maximum over ranks. backend "nccl" (RCCL over xGMI) on the GPU box, "gloo" in the CPU
tests -- the code path is the same.
"""


def shard_slice(rank: int, per_rank: int):
    """[start, stop) of this rank's reactors."""
    return rank * per_rank, (rank + 1) * per_rank


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """The slowest rank's time (the bench contract: max over ranks)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_ensemble(U, stats, dist=None):
    """All-gather this rank's final states U[N, n] and stats[N, k] (torch tensors on the rank's
    device: HIP for nccl, CPU for gloo) into [W*N, n] / [W*N, k] in ensemble order."""
    import torch
    payload = torch.cat([U, stats], dim=1).contiguous()
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        out = payload
    else:
        parts = [torch.empty_like(payload) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, payload)
        out = torch.cat(parts, dim=0)
    n = U.shape[1]
    return out[:, :n], out[:, n:]
