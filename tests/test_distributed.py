"""N>1 path on the CPU: world_size-2 ``gloo`` process groups.

The multi-GPU code (npe_pfn/distributed.py) is run for real -- its shard bounds, its
all_to_all of target tokens, its all_gathers, its Philox row bookkeeping and its counter
agreement -- with CPU stand-ins only where the GPU would compute:

* ``StubEngine`` honours the engine contract the estimator-parallel loop relies on
  (include/npfn.h npfn_set_estimator_range / npfn_forward_targets / npfn_head_sample):
  a target token depends on (global estimator, row, features) only, a draw on (all
  estimators' tokens of the row, global Philox row, counter) only.  The 2-rank
  ``ep_ar_sample`` must then equal the 1-process loop bit for bit -- the property the
  real kernels give (checked on the GPU in tests/test_gpu_multigpu.py).
* ``StubPosterior`` draws are a pure function of (observation, global Philox row).

The process group is set up through a file store (no port race).
"""
import os
import tempfile
from types import SimpleNamespace

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class StubEngine:
    """CPU stand-in with the estimator-parallel surface of npe_pfn.engine.Engine."""

    def __init__(self, n_estimators=4, d=8):
        self.cfg = SimpleNamespace(n_estimators=n_estimators, d_model=d)
        self.device = torch.device("cpu")
        self.e0, self.ne, self.es = 0, n_estimators, 1
        self.fits = 0

    def set_estimator_set(self, e0, count, stride):
        self.e0, self.ne, self.es = e0, count, stride

    def fit(self, X, y):
        self.ystat = float(y.double().mean()) + 0.01 * X.shape[1]
        self.fits += 1

    def ar_fit_begin(self, x_ctx, theta_ctx):  # npfn_ar_fit_begin / npfn_ar_fit_step
        self._joint = torch.cat([x_ctx, theta_ctx], 1)
        self._dx = x_ctx.shape[1]

    def ar_fit_step(self, k):
        F = self._dx + k
        self.fit(self._joint[:, :F], self._joint[:, F])

    def forward_targets(self, Xq):
        e = (self.e0 + self.es * torch.arange(self.ne, dtype=torch.float64))[:, None, None]
        j = torch.arange(self.cfg.d_model, dtype=torch.float64)[None, None, :]
        rowv = Xq.double().sum(1)[None, :, None]
        return (torch.sin(e + 0.1 * j) * rowv + self.ystat).to(torch.bfloat16)

    def head_sample(self, tokens, counter, row_base=0, log_prob_acc=None, eps=1e-15):
        assert tokens.shape[0] == self.cfg.n_estimators and tokens.dtype == torch.bfloat16
        n = tokens.shape[1]
        g = torch.arange(row_base, row_base + n, dtype=torch.float64)
        w = torch.arange(1, tokens.shape[0] + 1, dtype=torch.float64)[:, None]
        th = (tokens.double().sum(2) * w).sum(0) * 1e-3 + torch.sin(g * 0.37 + counter)
        if log_prob_acc is not None:
            log_prob_acc += th.float() * 0.5
        return th.float()


class StubPosterior:
    """sample_batched / _sample_impl draws depend on the observation value and the global row only."""

    def __init__(self, dth=3, seed=0):
        self._theta_train = torch.zeros(5, dth)
        self._obs_offset = 0
        self.seed = seed
        self._model = SimpleNamespace(sample_counter=0)

    def _rows(self, x, n):
        n_obs = x.shape[0]
        g = (self._obs_offset + torch.arange(n_obs))[:, None] * n + torch.arange(n)[None, :]  # global rows
        base = torch.sin(g.double() * 0.37 + self.seed)[..., None] + torch.arange(self._theta_train.shape[1])
        return (base + x[:, None, :1].double()).float()

    def sample_batched(self, x, sample_shape, with_log_prob=False):
        n = torch.Size(sample_shape).numel()
        th = self._rows(x, n)
        return (th, th.sum(-1)) if with_log_prob else th

    def sample(self, sample_shape, x=None):
        n = torch.Size(sample_shape).numel()
        return torch.full((n, self._theta_train.shape[1]), float(self.seed))

    def _sample_impl(self, sample_shape, x, max_sampling_batch_size, with_log_prob, eps, max_iter_rejection,
                     row_base_of=None, ar=None):
        n = torch.Size(sample_shape).numel()
        rb = row_base_of(0) if row_base_of else 0
        th = torch.sin((rb + torch.arange(n)).double()[:, None] * 0.37 + torch.arange(3)).float()
        return (th, th.sum(1)) if with_log_prob else th


def _ep_inputs():
    g = torch.Generator().manual_seed(0)
    x_ctx, th_ctx = torch.randn(20, 3, generator=g), torch.randn(20, 2, generator=g)
    xq = torch.randn(1, 3, generator=g).repeat(11, 1) + 0.1 * torch.randn(11, 3, generator=g)
    return x_ctx, th_ctx, xq


def _by_value(obj, to_np=True):
    """Tensors -> numpy (and back): results cross the queue BY VALUE -- a torch tensor would
    travel as a shared-memory handle that the parent opens through the child's resource
    sharer, which is gone once the child has exited (the race that made this fixture flaky)."""
    if isinstance(obj, torch.Tensor) and to_np:
        t = obj.detach().cpu()
        return ("__t__", (t.view(torch.int16) if t.dtype == torch.bfloat16 else t).numpy(), str(t.dtype))
    if isinstance(obj, tuple) and len(obj) == 3 and obj[0] == "__t__" and not to_np:
        import numpy as np

        t = torch.from_numpy(np.array(obj[1]))
        return t.view(torch.bfloat16) if obj[2] == "torch.bfloat16" else t
    if isinstance(obj, dict):
        return {k: _by_value(v, to_np) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_by_value(v, to_np) for v in obj)
    return obj


def _worker(rank, world, init_file, q):
    try:
        _worker_body(rank, world, init_file, q)
    except BaseException as e:  # report instead of dying silently (the parent's q.get would fail obscurely)
        import traceback

        q.put((rank, {"error": traceback.format_exc()}))
        raise


def _worker_body(rank, world, init_file, q):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    try:
        from npe_pfn.distributed import (all_gather_rows, ep_ar_sample, exchange_targets, sample_batched_sharded,
                                         sample_replicas, sample_rows_sharded, shard_bounds)

        res = {}
        for n_obs in (4, 3, 1):
            x = torch.arange(n_obs * 2, dtype=torch.float32).reshape(n_obs, 2)
            post = StubPosterior()
            th, lp = sample_batched_sharded(post, x, (6,), with_log_prob=True)
            res[n_obs] = (th, lp)
            assert post._obs_offset == 0
        # variable-length gather with lengths exchanged on the fly
        t = torch.full((rank + 1, 2), float(rank))
        res["rows"] = all_gather_rows(t)
        res["rep"] = sample_replicas(StubPosterior(seed=rank), torch.zeros(1, 2), 4)
        res["bounds"] = [shard_bounds(5, r, world) for r in range(world)]
        # estimator-parallel loop (11 rows: unequal row shards 6 / 5)
        eng = StubEngine()
        x_ctx, th_ctx, xq = _ep_inputs()
        res["ep"] = ep_ar_sample(eng, x_ctx, th_ctx, xq, counter=7, with_log_prob=True)
        res["ep_set"] = (eng.e0, eng.ne, eng.es)
        # repeated query rows: step 0 forwards the distinct row once and hands it to every row
        xu = xq[:1]
        res["ep_rep"] = ep_ar_sample(StubEngine(), x_ctx, th_ctx, xu.repeat(11, 1), counter=7, with_log_prob=True,
                                     x_unique=xu)
        # the all_to_all alone: rank r receives every estimator's tokens of its rows
        from npe_pfn.distributed import collective_stats

        collective_stats(reset=True)
        tok = torch.arange(2 * 11 * 4, dtype=torch.float32).reshape(2, 11, 4).add(100 * rank).to(torch.bfloat16)
        res["x2"] = exchange_targets(tok, 11)
        all_gather_rows(torch.zeros(3, 2), n_total=5)
        res["coll"] = collective_stats()
        # row-sharded sample with counter agreement (rank 1 ran one more accept/reject round)
        post = StubPosterior()
        post._model.sample_counter = 10 + 3 * rank
        res["rowshard"] = sample_rows_sharded(post, torch.zeros(1, 2), (9,), with_log_prob=True)
        res["counter"] = post._model.sample_counter
        q.put((rank, _by_value(res)))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def results():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        init_file = os.path.join(d, "pg")
        procs = [ctx.Process(target=_worker, args=(r, world, init_file, q)) for r in range(world)]
        for p in procs:
            p.start()
        out = {r: _by_value(res, False) for r, res in (q.get(timeout=180) for _ in range(world))}
        for r, res in out.items():
            assert "error" not in res, res.get("error")
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    return out


@pytest.mark.parametrize("n_obs", [4, 3, 1])
def test_sharded_sample_batched_equals_unsharded(results, n_obs):
    x = torch.arange(n_obs * 2, dtype=torch.float32).reshape(n_obs, 2)
    th_ref, lp_ref = StubPosterior().sample_batched(x, (6,), with_log_prob=True)
    for rank in (0, 1):
        th, lp = results[rank][n_obs]
        assert th.shape == (n_obs, 6, 3)
        assert torch.equal(th, th_ref) and torch.equal(lp, lp_ref)


def test_all_gather_variable_rows(results):
    want = torch.cat([torch.full((1, 2), 0.0), torch.full((2, 2), 1.0)])
    for rank in (0, 1):
        assert torch.equal(results[rank]["rows"], want)


def test_replicas_gather_in_rank_order(results):
    want = torch.cat([torch.zeros(4, 3), torch.ones(4, 3)])
    assert torch.equal(results[0]["rep"], want) and torch.equal(results[1]["rep"], want)


def test_shard_bounds_cover_range(results):
    assert results[0]["bounds"] == [(0, 3), (3, 5)]
    from npe_pfn.distributed import shard_bounds

    for n in (0, 1, 7, 64):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))


def test_estimator_parallel_equals_single_process(results):
    """2 ranks x 2 estimators (strided sets {0, 2}, {1, 3}) == 1 process x 4 estimators, bit
    for bit, on every rank."""
    from npe_pfn.distributed import ep_ar_sample

    x_ctx, th_ctx, xq = _ep_inputs()
    th_ref, lp_ref = ep_ar_sample(StubEngine(), x_ctx, th_ctx, xq, counter=7, with_log_prob=True)
    assert th_ref.shape == (11, 2) and lp_ref.shape == (11,)
    for rank in (0, 1):
        th, lp = results[rank]["ep"]
        assert torch.equal(th, th_ref) and torch.equal(lp, lp_ref)
    assert results[0]["ep_set"] == (0, 2, 2) and results[1]["ep_set"] == (1, 2, 2)


def test_estimator_parallel_repeated_rows(results):
    """x_unique (step 0 over the distinct rows, tokens handed to every row) == the loop over the
    repeated rows, on 2 ranks and in one process."""
    from npe_pfn.distributed import ep_ar_sample

    x_ctx, th_ctx, xq = _ep_inputs()
    xu = xq[:1]
    th_ref, lp_ref = ep_ar_sample(StubEngine(), x_ctx, th_ctx, xu.repeat(11, 1), counter=7, with_log_prob=True)
    th_u, lp_u = ep_ar_sample(StubEngine(), x_ctx, th_ctx, xu.repeat(11, 1), counter=7, with_log_prob=True,
                              x_unique=xu)
    assert torch.equal(th_u, th_ref) and torch.equal(lp_u, lp_ref)
    for rank in (0, 1):
        th, lp = results[rank]["ep_rep"]
        assert torch.equal(th, th_ref) and torch.equal(lp, lp_ref)


def test_exchange_targets_layout(results):
    """Rank r gets [E=4, rows of r, d]: estimators 0-1 from rank 0, 2-3 from rank 1."""
    full = torch.cat([torch.arange(2 * 11 * 4, dtype=torch.float32).reshape(2, 11, 4).add(100 * r)
                      for r in (0, 1)]).to(torch.bfloat16)
    assert torch.equal(results[0]["x2"], full[:, :6]) and torch.equal(results[1]["x2"], full[:, 6:])


def test_rows_sharded_draws_unsharded_rows_and_agrees_counter(results):
    th_ref = torch.sin(torch.arange(9).double()[:, None] * 0.37 + torch.arange(3)).float()
    for rank in (0, 1):
        th, lp = results[rank]["rowshard"]
        assert torch.equal(th, th_ref) and torch.equal(lp, th_ref.sum(1))
        assert results[rank]["counter"] == 13


def test_canonical_order_and_layout():
    from npe_pfn.distributed import canonical_order, ep_layout

    # rank-major tokens of strided sets, 2 ranks x 3 estimators: rank r holds r, r+2, r+4
    rm = torch.tensor([0, 2, 4, 1, 3, 5])
    assert torch.equal(canonical_order(rm, 2), torch.arange(6))
    assert ep_layout(8, 8) == (4, 2) and ep_layout(4, 8) == (4, 1) and ep_layout(2, 8) == (2, 1)
    assert ep_layout(8, 8, max_ep=8) == (8, 1) and ep_layout(3, 8) == (1, 3) and ep_layout(1, 8) == (1, 1)


class HybridStubPosterior:
    """_sample_impl draws one batch through the ar hook; its query rows are a function of the
    global Philox row, so row groups must hand the hook the right row_base."""

    def __init__(self, eng):
        self._model = SimpleNamespace(engine=eng, sample_counter=3)
        self._theta_train = torch.zeros(20, 2)

    @staticmethod
    def inputs(rows):
        x_ctx, th_ctx, _ = _ep_inputs()
        g = rows.double()[:, None]
        return x_ctx, th_ctx, (torch.sin(g * 0.3 + torch.arange(3)) * 0.5).float()

    def _sample_impl(self, sample_shape, x, mbs, with_log_prob, eps, mir, row_base_of=None, ar=None):
        n = torch.Size(sample_shape).numel()
        rb = row_base_of(0) if row_base_of is not None else 0
        x_ctx, th_ctx, xq = self.inputs(torch.arange(rb, rb + n))
        return ar(x_ctx, th_ctx, xq, with_log_prob, eps, rb)


def _hybrid_worker(rank, world, init_file, q):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    try:
        from npe_pfn.distributed import sample_estimator_parallel

        post = HybridStubPosterior(StubEngine())
        th, lp = sample_estimator_parallel(post, torch.zeros(1, 3), (13,), with_log_prob=True, ep_size=2)
        q.put((rank, _by_value((th, lp, post._model.engine.e0, post._model.engine.es, post._model.sample_counter))))
    finally:
        dist.destroy_process_group()


def test_ep_groups_times_row_groups_equal_single_process():
    """4 ranks = 2 EP groups (strided sets of 2 estimators) x 2 row groups (7 + 6 rows): every
    rank returns the 13 rows of the 1-process loop, bit for bit."""
    from npe_pfn.distributed import ep_ar_sample

    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        init_file = os.path.join(d, "pg")
        procs = [ctx.Process(target=_hybrid_worker, args=(r, world, init_file, q)) for r in range(world)]
        for p in procs:
            p.start()
        out = {r: _by_value(res, False) for r, res in (q.get(timeout=180) for _ in range(world))}
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    x_ctx, th_ctx, xq = HybridStubPosterior.inputs(torch.arange(13))
    th_ref, lp_ref = ep_ar_sample(StubEngine(), x_ctx, th_ctx, xq, counter=3, with_log_prob=True)
    for r in range(world):
        th, lp, e0, es, counter = out[r]
        assert torch.equal(th, th_ref) and torch.equal(lp, lp_ref)
        assert (e0, es) == (r % 2, 2) and counter == 5


def test_collective_byte_accounting(results):
    """bench.py's per-step collective bytes at N > 1: the all_to_all sends this rank's whole
    [rows, E_loc * d] token block (11 x 2 x 4 bf16 = 176 B), the all_gather the padded shard
    (3 x 2 f32 = 24 B)."""
    for rank in (0, 1):
        c = results[rank]["coll"]
        assert c["all_to_all"] == {"calls": 1, "bytes": 176}
        assert c["all_gather"] == {"calls": 1, "bytes": 24}
