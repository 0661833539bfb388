"""The two multi-GPU forms of ONE ``TabPFN_Based_NPE_PFN.sample`` call give the same draws
(BASELINE.json north_star "single RCCL gather").

``bench.py --gpus N`` times the default estimator-parallel form (``sample_estimator_parallel``:
EP groups x row groups, one all_to_all + one all_gather per AR step) and, beside it in the same
JSON line (``alt_modes.rows``), the north_star form (``sample_rows_sharded``: replicated fit, row
shards, one all_gather at the end).  Here both run for real through ``gloo`` at world 2 and 4 on
the CPU -- the reference orchestration (``NPE_PFN_Core._sample_impl`` -> accept/reject ->
``_sample`` -> the AR hook), the shard bounds, the collectives and the Philox row and counter
bookkeeping -- with tests/test_distributed.py's ``StubEngine`` in place of the HIP engine (a
target token depends on (global estimator, row, features) only, a draw on (all estimators'
tokens of the row, global Philox row, counter) only: the property the kernels give, checked on
the GPU by tests/test_gpu_multigpu.py).  Both forms must equal the 1-process ``sample`` bit for
bit on every rank.  The prior is Gaussian (c2's: support R^d), so one accept/reject batch, as at
c2; under a box prior the forms' later batches draw at different Philox rows by design (each
row group's batches i > 0 sit at rows no other group uses).
"""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_distributed import StubEngine, _by_value


class ArStubEngine(StubEngine):
    """StubEngine plus the 1-process fused entry point (Engine.ar_sample's contract)."""

    ep_set = None

    def full_range(self):
        self.set_estimator_set(0, self.cfg.n_estimators, 1)
        self.ep_set = None

    def set_fit_token(self, tok):
        pass

    def ar_sample(self, x_ctx, theta_ctx, x_query, counter, with_log_prob=False, eps=1e-15, row_base=0,
                  x_unique=None):
        self.full_range()
        self.ar_fit_begin(x_ctx.float(), theta_ctx.float())
        feat = x_query.float()
        lp = torch.zeros(feat.shape[0]) if with_log_prob else None
        cols = []
        for k in range(theta_ctx.shape[1]):
            self.ar_fit_step(k)
            th = self.head_sample(self.forward_targets(feat), counter + k, row_base=row_base, log_prob_acc=lp,
                                  eps=eps)
            cols.append(th[:, None])
            feat = torch.cat([feat, th[:, None]], 1)
        return torch.cat(cols, 1), lp


def _posterior():
    from npe_pfn.npe_pfn import TabPFN_Based_NPE_PFN

    g = torch.Generator().manual_seed(5)
    theta, x = torch.randn(40, 2, generator=g), torch.randn(40, 3, generator=g)
    prior = torch.distributions.Independent(torch.distributions.Normal(torch.zeros(2), torch.ones(2)), 1)
    post = TabPFN_Based_NPE_PFN(prior=prior, regressor_init_kwargs={"random_state": 4, "n_estimators": 4})
    post._model._engine = ArStubEngine(n_estimators=4)
    post.append_simulations(theta, x)
    return post, x[:1] + 0.05


N = 23


def _worker(rank, world, init_file, q):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    try:
        from npe_pfn.distributed import collective_stats, sample_estimator_parallel, sample_rows_sharded

        post, x_o = _posterior()
        c0 = post._model.sample_counter
        collective_stats(reset=True)
        ep = sample_estimator_parallel(post, x_o, (N,), with_log_prob=True)
        ep_coll = collective_stats()
        c_ep = post._model.sample_counter
        post._model.sample_counter = c0
        rows = sample_rows_sharded(post, x_o, (N,), with_log_prob=True)
        rows_coll = collective_stats()
        q.put((rank, _by_value({"ep": ep, "rows": rows, "c_ep": c_ep, "c_rows": post._model.sample_counter,
                                "ep_coll": ep_coll, "rows_coll": rows_coll})))
    except BaseException:
        import traceback

        q.put((rank, {"error": traceback.format_exc()}))
        raise
    finally:
        dist.destroy_process_group()


def _run(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        init_file = os.path.join(d, "pg")
        procs = [ctx.Process(target=_worker, args=(r, world, init_file, q)) for r in range(world)]
        for p in procs:
            p.start()
        out = {r: _by_value(res, False) for r, res in (q.get(timeout=240) for _ in range(world))}
        for p in procs:
            p.join(timeout=60)
        for r, res in out.items():
            assert "error" not in res, res.get("error")
        assert all(p.exitcode == 0 for p in procs)
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_ep_and_rows_forms_draw_the_single_process_sample(world):
    post, x_o = _posterior()
    th_ref, lp_ref = post.sample((N,), x=x_o, with_log_prob=True)
    assert th_ref.shape == (N, 2)
    out = _run(world)
    for r in range(world):
        (th_ep, lp_ep), (th_rows, lp_rows) = out[r]["ep"], out[r]["rows"]
        assert torch.equal(th_ep, th_ref) and torch.equal(lp_ep, lp_ref), f"EP form, rank {r}"
        assert torch.equal(th_rows, th_ref) and torch.equal(lp_rows, lp_ref), f"rows form, rank {r}"
        # both forms leave every rank at the counter of the 1-process call (2 AR dims, one batch)
        assert out[r]["c_ep"] == out[r]["c_rows"] == post._model.sample_counter == 2
        # the north_star form: no per-step exchange, the gathers at the end only
        assert "all_to_all" not in out[r]["rows_coll"]
        assert out[r]["ep_coll"]["all_to_all"]["calls"] == 2  # one per AR step
