"""N>1 path on the CPU: world_size-2 ``gloo`` process groups.

The sharding helpers (npe_pfn/distributed.py) must return, on every rank, exactly
what one process computes for the whole batch.  The posterior here is a stub
whose draws are a pure function of (observation, global Philox row) -- the
contract the engine honours through ``NPE_PFN_Core._obs_offset`` /
``npfn_ar_sample(row_base)`` (checked on the GPU in test_gpu_sharding.py).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class StubPosterior:
    """sample_batched draws depend on the observation value and the global row index only."""

    def __init__(self, dth=3, seed=0):
        self._theta_train = torch.zeros(5, dth)
        self._obs_offset = 0
        self.seed = seed

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


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from npe_pfn.distributed import all_gather_rows, sample_batched_sharded, sample_replicas, shard_bounds

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
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def results():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
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
