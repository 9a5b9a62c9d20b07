"""Ray-batch sharding across GPUs (one process per GPU, torch.distributed over RCCL).

The reference runs independent single-ray processes and merges files afterwards
(runner_example.sh:4-7, Combine_Files.py). Here a global batch of rays is split into
contiguous blocks of global ray ids, one per rank. The sampler's Philox stream is keyed
by the *global* id, so the batch does not depend on the GPU count. The only data-path
collective is the sum of the binned flux (plot/flux.py:38-48). The run's totals
(Σ ray-steps, Σ rays) are summed and the wall time is max-reduced, for the bench line.
"""
from __future__ import annotations


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """[lo, hi) of the global ray ids owned by `rank`: contiguous, sizes differ by at most 1."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    return n_total * rank // world, n_total * (rank + 1) // world


def allreduce_flux(hist, world: int):
    """In-place sum of the per-rank flux histograms: one all-reduce of 2 x nbins f64 (RCCL
    on GPU tensors, gloo on CPU tensors)."""
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(hist)
    return hist


def allreduce_sum(values):
    """Element-wise sum of a float64 vector over all ranks (torch.distributed: RCCL on the GPU
    for the nccl backend, gloo on the CPU). Returns a numpy array."""
    import numpy as np
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.as_tensor(np.asarray(values, np.float64)).to(dev)
    dist.all_reduce(t)
    return t.cpu().numpy()


def reduce_totals(steps: float, elapsed_s: float, rays: int, world: int, device=None):
    """(Σ steps, max wall time, Σ rays) over ranks."""
    import torch
    import torch.distributed as dist
    s = torch.tensor([float(steps), float(rays)], dtype=torch.float64, device=device)
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(s)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(s[0]), float(t[0]), int(round(float(s[1])))
