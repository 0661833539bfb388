"""Multi-GPU posterior sampling.

One process per GPU (``torch.distributed``; backend ``"nccl"`` is RCCL over xGMI on
ROCm, ``"gloo"`` on the CPU for tests).  Three ways to split the work:

* :func:`sample_estimator_parallel` -- strong scaling of ONE ``sample((N,), x_o)`` call
  (c2, c3; the bench's default at N > 1).  The ranks form EP groups of g ranks
  (:func:`ep_layout`); rank j of a group owns the strided estimator set
  ``{j, j+g, j+2g, ...}`` of the ensemble (``npfn_set_estimator_set``) and, per
  autoregressive step, fits them (train-side forward: 1/g of the fit work) and runs
  their test-side forward over the group's query rows.  One ``all_to_all`` then hands
  every rank the decoder-input target tokens of ALL estimators for its row shard (E x N/g x
  192 bf16: 3.8 MB at c2 and g = 8), reordered to estimator order, the rank runs the
  decoder head, ensemble mix and bar sample for those rows (``npfn_head_sample``, Philox
  rows = global rows), and one ``all_gather`` of the sampled column (N floats) gives every
  rank of the group the next step's feature table.  The draws are bit for bit the 1-GPU
  draws (a row's arithmetic does not depend on which estimators or rows share its launch:
  npfn_rowk2.hip per-estimator tiles, npfn_engine.hip decode_chunk).  Strided sets keep the
  groups balanced: in tabpfn's ensemble the estimators 0-3 (quantile + SVD features) carry
  about 2x the tokens of 4-7 (Yeo-Johnson), so a contiguous split would leave half the ranks
  idle half the time.  With more ranks than balanced EP allows (8 ranks, 8 estimators of
  two kinds), the ranks form ``world / g`` ROW GROUPS: each draws its quota of the N rows
  as :func:`sample_rows_sharded` does, estimator-parallel inside, and the groups' rows are
  gathered at the end (the fit is replicated across row groups only).
* :func:`sample_rows_sharded` -- the row split of §8e: rank r draws its quota of rows
  ``[r N/G, (r+1) N/G)`` with the fit replicated on every rank, then one ``all_gather``.
  The first accept/reject batch draws at the unsharded Philox rows (row_base = r N/G);
  later batches (box priors) draw at rank-disjoint rows.
* :func:`sample_batched_sharded` -- c5: observations are split into contiguous shards,
  rank r samples its shard with ``sample_batched`` (Philox rows of the unsharded
  obs-major batch, ``_obs_offset``) and the shards are gathered in observation order.
* :func:`sample_replicas` -- weak-scaling replicas (every rank its own n draws), kept as
  an explicitly labelled secondary mode of bench.py.

After a sharded call every rank's ``sample_counter`` is set to the maximum over ranks
(ranks whose shard filled in fewer accept/reject rounds would otherwise fall behind and
draw other Philox streams on the next call).
"""

from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist
from torch import Tensor

__all__ = ["shard_bounds", "all_gather_rows", "sample_estimator_parallel", "ep_ar_sample", "ep_layout",
           "canonical_order", "sample_rows_sharded", "sample_batched_sharded", "sample_replicas", "sync_sample_counter",
           "phase_timing", "phase_timing_read", "collective_stats"]

# Per-phase timing of ep_ar_sample (bench.py's per_rank split at N > 1): while enabled, every AR
# step records device events around its phases on the current stream -- compute (fit step +
# forward_targets), exchange (all_to_all of target tokens; the current stream waits for the
# collective), head (decoder + mix + bar sample), gather (all_gather of the sampled column).
# Resolved only by phase_timing_read(), so the timed loop never synchronises for it.
_PHASES = ("compute", "exchange", "head", "gather")
_TIMING = {"on": False, "events": []}


def phase_timing(on: bool = True) -> None:
    _TIMING["on"] = bool(on)
    _TIMING["events"] = []


def phase_timing_read() -> dict:
    """{phase: ms} summed over the recorded steps (synchronises), plus "steps"."""
    out = {p: 0.0 for p in _PHASES}
    evs = _TIMING["events"]
    if evs:
        evs[-1][-1].synchronize()
    for e in evs:
        for i, p in enumerate(_PHASES):
            out[p] += e[i].elapsed_time(e[i + 1])
    out["steps"] = len(evs)
    _TIMING["events"] = []
    return out


# Bytes this rank puts into each kind of collective (send side), for bench.py's per-step
# accounting at N > 1: {kind: [calls, bytes]}; collective_stats(reset=True) reads and clears.
_COLL = {}


def _count(kind: str, nbytes: int) -> None:
    c = _COLL.setdefault(kind, [0, 0])
    c[0] += 1
    c[1] += int(nbytes)


def collective_stats(reset: bool = True) -> dict:
    out = {k: {"calls": v[0], "bytes": v[1]} for k, v in _COLL.items()}
    if reset:
        _COLL.clear()
    return out


def _mark():
    if not _TIMING["on"] or not torch.cuda.is_available():
        return None
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    return ev


def _rank_world(group=None) -> Tuple[int, int]:
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def _comm_device(t: Tensor, group=None) -> torch.device:
    """Where a collective on ``t`` runs: its own device, except CUDA tensors under gloo (the
    CPU rehearsal of the multi-GPU path on one GPU), which travel through host copies."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        return torch.device("cpu")
    return t.device


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
    home = t.device
    t = t.to(_comm_device(t, group)).contiguous()
    if n_total is None:
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
        ns = torch.empty(world, dtype=torch.int64, device=t.device)
        dist.all_gather_into_tensor(ns, n, group=group)
        _count("all_gather", n.numel() * n.element_size())
        lens = [int(v) for v in ns.cpu()]
    else:
        lens = [b - a for a, b in (shard_bounds(n_total, r, world) for r in range(world))]
    m = max(lens)
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    out = torch.empty((world * m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    _count("all_gather", pad.numel() * pad.element_size())
    return torch.cat([out[r * m: r * m + lens[r]] for r in range(world)], 0).to(home)


def sync_sample_counter(regressor, group=None) -> None:
    """Every rank continues from the largest Philox step counter any rank reached."""
    rank, world = _rank_world(group)
    if world == 1 or regressor is None or not hasattr(regressor, "sample_counter"):
        return
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    c = torch.tensor([int(regressor.sample_counter)], dtype=torch.int64, device=dev)
    dist.all_reduce(c, op=dist.ReduceOp.MAX, group=group)
    _count("all_reduce", c.numel() * c.element_size())
    regressor.sample_counter = int(c.item())


# ----------------------------------------------------------- estimator-parallel
def exchange_targets(tok: Tensor, n_rows: int, group=None) -> Tensor:
    """[E_loc, N, d] target tokens of this rank's estimators -> [E, n_r, d] tokens of ALL
    estimators for this rank's row shard, in rank-major order (one all_to_all;
    :func:`canonical_order` restores estimator order for strided sets)."""
    rank, world = _rank_world(group)
    e_loc, n, d = tok.shape
    assert n == n_rows
    if world == 1:
        return tok
    bounds = [shard_bounds(n, r, world) for r in range(world)]
    a, b = bounds[rank]
    # rows-major so that each destination's rows are one contiguous block; the 2-byte tokens
    # travel as int32 pairs (a pure byte move, no reduction; gloo has no 16-bit all_to_all)
    assert (e_loc * d * tok.element_size()) % 4 == 0
    w = e_loc * d * tok.element_size() // 4
    cdev = _comm_device(tok, group)
    send = tok.transpose(0, 1).contiguous().view(torch.int32).reshape(n, w).to(cdev)
    recv = torch.empty((world * (b - a), w), dtype=torch.int32, device=cdev)
    dist.all_to_all_single(recv, send, output_split_sizes=[b - a] * world,
                           input_split_sizes=[hi - lo for lo, hi in bounds], group=group)
    _count("all_to_all", send.numel() * send.element_size())
    out = recv.view(tok.dtype).view(world, b - a, e_loc, d).permute(0, 2, 1, 3).reshape(world * e_loc, b - a, d)
    return out.contiguous().to(tok.device)


def ep_layout(world: int, n_estimators: int, max_ep: Optional[int] = None) -> Tuple[int, int]:
    """(g, row_groups): EP group size and number of row groups for ``world`` ranks -- the
    largest divisor g of ``world`` that divides ``n_estimators`` and is at most ``max_ep``
    (default: n_estimators // 2, so that a strided set holds estimators of both halves of
    the ensemble), ``world // g`` row groups."""
    cap = n_estimators // 2 if max_ep is None else int(max_ep)
    g = 1
    for d in range(1, world + 1):
        if world % d == 0 and n_estimators % d == 0 and d <= max(cap, 1):
            g = d
    return g, world // g


def canonical_order(tok: Tensor, world: int) -> Tensor:
    """[E, ...] tokens in rank-major order of strided sets (rank r: estimators r, r+g, ...) ->
    estimator order."""
    E = tok.shape[0]
    e_loc = E // world
    return tok.view(world, e_loc, *tok.shape[1:]).transpose(0, 1).reshape(tok.shape).contiguous()


def ep_ar_sample(engine, x_ctx: Tensor, theta_ctx: Tensor, x_query: Tensor, counter: int,
                 with_log_prob: bool = False, eps: float = 1e-15, group=None,
                 row_base: int = 0, x_unique: Optional[Tensor] = None) -> Tuple[Tensor, Optional[Tensor]]:
    """The autoregressive dimension loop (npe_pfn.py:135-169) split by estimator over the
    ranks of ``group``.

    ``engine`` offers ``set_estimator_set``, ``ar_fit_begin`` / ``ar_fit_step`` (or ``fit``),
    ``forward_targets`` and ``head_sample`` (npe_pfn.engine.Engine).  ``row_base`` = Philox row of the first query
    row.  Returns the full ``[N, dθ]`` draws (and ``[N]`` log-probs) on every rank of the
    group, equal bit for bit to ``engine.ar_sample`` on one GPU.  ``x_unique``: the distinct rows
    ``x_query`` repeats (obs-major); step 0 then runs the forward once per distinct row and
    hands each query row its row's tokens, as ``engine.ar_sample(..., x_unique=...)`` does.
    """
    rank, world = _rank_world(group)
    E = engine.cfg.n_estimators
    if E % world:
        raise ValueError(f"estimator-parallel sampling needs world size | n_estimators ({world} vs {E})")
    e_loc = E // world
    if getattr(engine, "ep_set", None) != (rank, e_loc, world):
        engine.set_estimator_set(rank, e_loc, world)
        engine.ep_set = (rank, e_loc, world)  # kept across the accept/reject batches of one call
    dev = engine.device
    x_ctx = x_ctx.to(dev, torch.float32)
    theta_ctx = theta_ctx.to(dev, torch.float32)
    feat = x_query.to(dev, torch.float32).contiguous()
    n, dx = x_ctx.shape
    dth = theta_ctx.shape[1]
    N = feat.shape[0]
    joint = torch.cat([x_ctx, theta_ctx], 1).contiguous()
    a, b = shard_bounds(N, rank, world)
    lp = torch.zeros(b - a, dtype=torch.float32, device=dev) if with_log_prob else None
    cols: List[Tensor] = []
    stepwise = hasattr(engine, "ar_fit_begin")
    if stepwise:  # every step's preprocessing fit queued at once, reused across batches (fit token)
        engine.ar_fit_begin(x_ctx, theta_ctx)
    for k in range(dth):
        m0 = _mark()
        if stepwise:
            engine.ar_fit_step(k)
        else:
            engine.fit(joint[:, : dx + k], joint[:, dx + k])
        if k == 0 and x_unique is not None:
            U = x_unique.shape[0]
            idx = torch.arange(N, device=dev) // (N // U)
            tok = engine.forward_targets(x_unique.to(dev, torch.float32)).index_select(1, idx)
        else:
            tok = engine.forward_targets(feat)
        m1 = _mark()
        mine = canonical_order(exchange_targets(tok, N, group), world)
        m2 = _mark()
        th = engine.head_sample(mine, counter + k, row_base=row_base + a, log_prob_acc=lp, eps=eps)
        m3 = _mark()
        col = all_gather_rows(th[:, None], n_total=N, group=group)
        m4 = _mark()
        if m0 is not None:
            _TIMING["events"].append((m0, m1, m2, m3, m4))
        cols.append(col)
        feat = torch.cat([feat, col], 1)
    theta = torch.cat(cols, 1)
    if with_log_prob:
        lp = all_gather_rows(lp, n_total=N, group=group)
    return theta, lp


_GROUPS = {}


def ep_groups(g: int, group=None):
    """(ep_group, peer_group, row_group_index) of this rank for EP groups of g consecutive
    ranks; peers = the ranks with the same index in every EP group.  Created once per layout
    (torch.distributed.new_group is collective: every rank creates every group)."""
    rank, world = _rank_world(group)
    if g == world:
        return group, None, 0
    if world % g:
        raise ValueError(f"EP group size {g} does not divide the world size {world}")
    # ranks of `group` as global ranks (new_group takes global ranks)
    glob = [dist.get_global_rank(group, r) for r in range(world)] if group is not None else list(range(world))
    key = (g, world, tuple(glob))
    if key not in _GROUPS:
        eps_ = [dist.new_group([glob[r] for r in range(q * g, q * g + g)]) for q in range(world // g)]
        peers = [dist.new_group([glob[r] for r in range(j, world, g)]) for j in range(g)]
        _GROUPS[key] = (eps_, peers)
    eps_, peers = _GROUPS[key]
    return eps_[rank // g], peers[rank % g], rank // g


def sample_estimator_parallel(posterior, x: Tensor, sample_shape=torch.Size(), with_log_prob: bool = False,
                              eps: float = 1e-15, max_sampling_batch_size: int = 10_000,
                              max_iter_rejection: Optional[int] = None, group=None, ep_size: Optional[int] = None):
    """``posterior.sample(sample_shape, x)`` with every accept/reject batch's dimension loop
    split by estimator (:func:`ep_ar_sample`) inside EP groups of ``ep_size`` ranks (default:
    :func:`ep_layout`) and the rows split over the groups; the same result on every rank.
    With one group the draws equal the 1-GPU ``sample``."""
    reg = posterior._model
    eng = reg.engine
    rank, world = _rank_world(group)
    E = eng.cfg.n_estimators
    g = ep_layout(world, E)[0] if ep_size is None else int(ep_size)
    if g < 1 or world % g or E % g:
        raise ValueError(f"ep_size {g} must divide both the world size ({world}) and n_estimators ({E})")
    if g == 1 and world > 1:  # no estimator split: the plain row split (keeps the fit reuse)
        return sample_rows_sharded(posterior, x, sample_shape, with_log_prob, eps, max_sampling_batch_size,
                                   max_iter_rejection, group)
    ep_group, peer_group, q = ep_groups(g, group)
    try:
        return _sample_ep(posterior, reg, eng, x, sample_shape, with_log_prob, eps, max_sampling_batch_size,
                          max_iter_rejection, group, g, ep_group, peer_group, q, world)
    finally:
        # the posterior's other entry points (sample, log_prob, sample_batched) need the whole
        # ensemble on this engine again
        if hasattr(eng, "full_range"):
            eng.full_range()


def _sample_ep(posterior, reg, eng, x, sample_shape, with_log_prob, eps, max_sampling_batch_size, max_iter_rejection,
               group, g, ep_group, peer_group, q, world):

    def ar(x_ctx, theta_ctx, x_query, wlp, eps_, row_base=0, x_unique=None):
        counter = reg.sample_counter
        reg.sample_counter += int(theta_ctx.shape[1])
        return ep_ar_sample(eng, x_ctx, theta_ctx, x_query, counter, wlp, eps_, group=ep_group, row_base=row_base,
                            x_unique=x_unique)

    if peer_group is None:  # one EP group: every rank draws all rows
        return posterior._sample_impl(sample_shape, x, max_sampling_batch_size, with_log_prob, eps,
                                      max_iter_rejection, ar=ar)
    return _rows_over_groups(posterior, x, sample_shape, with_log_prob, eps, max_sampling_batch_size,
                             max_iter_rejection, q, world // g, peer_group, group, ar)


# ------------------------------------------------------------------- row split
def _rows_over_groups(posterior, x, sample_shape, with_log_prob, eps, max_sampling_batch_size, max_iter_rejection,
                      q: int, nq: int, peer_group, group, ar=None):
    """Row group q of nq draws rows ``[q N/nq, (q+1) N/nq)`` of one ``sample((N,))`` call (its
    first accept/reject batch at the unsharded Philox rows, later batches at rows no other
    group uses), then the groups' rows are gathered over ``peer_group`` in group order."""
    N = torch.Size(sample_shape).numel()
    a, b = shard_bounds(N, q, nq)

    def row_base_of(i: int) -> int:
        return a if i == 0 else N + ((i - 1) * nq + q) * max_sampling_batch_size

    if b > a:
        res = posterior._sample_impl((b - a,), x, max_sampling_batch_size, with_log_prob, eps, max_iter_rejection,
                                     row_base_of=row_base_of, ar=ar)
    else:
        dth = posterior._theta_train.shape[1]
        th0 = torch.empty((0, dth), device=x.device)
        res = (th0, torch.empty(0, device=x.device)) if with_log_prob else th0
    sync_sample_counter(getattr(posterior, "_model", None), group)
    th, lp = (res if with_log_prob else (res, None))
    th = all_gather_rows(th, n_total=N, group=peer_group)
    if with_log_prob:
        return th, all_gather_rows(lp, n_total=N, group=peer_group)
    return th


def sample_rows_sharded(posterior, x: Tensor, sample_shape=torch.Size(), with_log_prob: bool = False,
                        eps: float = 1e-15, max_sampling_batch_size: int = 10_000,
                        max_iter_rejection: Optional[int] = None, group=None):
    """Rank r draws rows ``[r N/G, (r+1) N/G)`` of one ``sample((N,))`` call (fit replicated),
    then one all_gather; every rank returns all N rows in rank order."""
    rank, world = _rank_world(group)
    return _rows_over_groups(posterior, x, sample_shape, with_log_prob, eps, max_sampling_batch_size,
                             max_iter_rejection, rank, world, group, group)


# ------------------------------------------------------------ observation split
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
    sync_sample_counter(getattr(posterior, "_model", None), group)
    th, lp = (res if with_log_prob else (res, None))
    th = all_gather_rows(th, n_total=n_obs, group=group)
    if with_log_prob:
        return th, all_gather_rows(lp, n_total=n_obs, group=group)
    return th


def sample_replicas(posterior, x: Tensor, n: int, group=None, **kwargs) -> Tensor:
    """Weak-scaling replicas: every rank draws ``n`` samples of the same observation; ``[world*n, dθ]``."""
    s = posterior.sample((n,), x=x, **kwargs)
    return all_gather_rows(s, group=group)
