"""Multi-GPU sharding of posterior sampling.

One process per GPU (``torch.distributed``; backend ``"nccl"`` is RCCL over
xGMI on ROCm, ``"gloo"`` on the CPU for tests).  Posterior rows are
independent through every autoregressive step, so the work shards with no
data-path collective; the only exchange is one all-gather of the results.

* :func:`sample_batched_sharded` -- c5: observations are split into
  contiguous shards, rank r samples its shard with ``sample_batched`` and the
  shards are gathered in observation order.  The engine draws the uniforms of
  a shard starting at the Philox row of its first observation in the
  unsharded obs-major batch (``NPE_PFN_Core._obs_offset``,
  ``npfn_ar_sample(row_base)``), so the gathered result equals the 1-GPU
  ``sample_batched`` of all observations.
* :func:`sample_replicas` -- c2 at N GPUs (weak scaling): every rank draws its
  own ``n`` samples for the same observation from its own Philox stream
  (``random_state`` = rank) and the samples are gathered.

The context fit is replicated on every rank (deterministic, same inputs);
SURVEY.md §8e notes the estimator-sharded alternative for strong scaling of
a single observation.
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist
from torch import Tensor

__all__ = ["shard_bounds", "all_gather_rows", "sample_batched_sharded", "sample_replicas"]


def _rank_world(group=None) -> Tuple[int, int]:
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def shard_bounds(n_items: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous near-equal split of ``range(n_items)``; the first ``n % world`` ranks get one more."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(int(n_items), world)
    a = rank * base + min(rank, extra)
    return a, a + base + (1 if rank < extra else 0)


def all_gather_rows(t: Tensor, n_total: Optional[int] = None, group=None) -> Tensor:
    """Concatenate every rank's ``t`` along dim 0 in rank order (shards may differ in length).

    One ``all_gather_into_tensor`` of the shards padded to the longest one (plus
    a tiny gather of the lengths when ``n_total`` is not given).
    """
    rank, world = _rank_world(group)
    if world == 1:
        return t
    t = t.contiguous()
    if n_total is None:
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
        ns = torch.empty(world, dtype=torch.int64, device=t.device)
        dist.all_gather_into_tensor(ns, n, group=group)
        lens = [int(v) for v in ns.cpu()]
    else:
        lens = [b - a for a, b in (shard_bounds(n_total, r, world) for r in range(world))]
    m = max(lens)
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    out = torch.empty((world * m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    return torch.cat([out[r * m: r * m + lens[r]] for r in range(world)], 0)


def sample_batched_sharded(posterior, x: Tensor, sample_shape=torch.Size(), with_log_prob: bool = False,
                           group=None, **kwargs):
    """``posterior.sample_batched(x, sample_shape)`` with the observations sharded over ranks.

    Returns the full ``[n_obs, n, dθ]`` result (and ``[n_obs, n]`` log-probs) on every rank.
    """
    rank, world = _rank_world(group)
    n_obs = x.shape[0]
    a, b = shard_bounds(n_obs, rank, world)
    n = torch.Size(sample_shape).numel()
    if b > a:
        posterior._obs_offset = a
        try:
            res = posterior.sample_batched(x[a:b], sample_shape, with_log_prob=with_log_prob, **kwargs)
        finally:
            posterior._obs_offset = 0
    else:  # more ranks than observations: this rank only joins the gather
        dth = posterior._theta_train.shape[1]
        th0 = torch.empty((0, n, dth), device=x.device)
        res = (th0, torch.empty((0, n), device=x.device)) if with_log_prob else th0
    th, lp = (res if with_log_prob else (res, None))
    th = all_gather_rows(th, n_total=n_obs, group=group)
    if with_log_prob:
        return th, all_gather_rows(lp, n_total=n_obs, group=group)
    return th


def sample_replicas(posterior, x: Tensor, n: int, group=None, **kwargs) -> Tensor:
    """Weak-scaling replicas: every rank draws ``n`` samples of the same observation; ``[world*n, dθ]``."""
    s = posterior.sample((n,), x=x, **kwargs)
    return all_gather_rows(s, group=group)
