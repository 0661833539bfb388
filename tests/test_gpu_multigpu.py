"""The estimator-parallel split of the AR loop on the engine (npe_pfn/distributed.py).

On one GPU, G simulated ranks each hold an engine restricted to the strided estimator set
{r, r+G, ...} (npfn_set_estimator_set; or the contiguous range [r E/G, (r+1) E/G),
npfn_set_estimator_range); per step every "rank" fits and runs npfn_forward_targets for its
estimators, the target tokens are exchanged by slicing and put back in estimator order
(what the all_to_all + canonical_order do), and each rank samples its row shard with
npfn_head_sample(row_base = first row).  The draws and log-probs must equal the 1-GPU
fused npfn_ar_sample BIT FOR BIT: a row's arithmetic does not depend on which
estimators or rows share a launch.
"""
import pytest
import torch

from npe_pfn.distributed import shard_bounds
from npe_pfn.tasks import gaussian_linear_prior, gaussian_linear_task
from npe_pfn.weights import ModelConfig, synthetic_weights

pytestmark = pytest.mark.gpu

CFG = ModelConfig()
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def weights():
    return synthetic_weights(CFG, seed=0)


@pytest.mark.parametrize("G,strided,pre,stepwise", [(2, True, "ensemble", True), (4, True, "ensemble", True),
                                                     (8, True, "ensemble", False), (2, False, "none", False),
                                                     (4, False, "ensemble", True)])
def test_estimator_parallel_split_is_bitwise_ar_sample(weights, G, strided, pre, stepwise):
    """stepwise: the ranks fit through npfn_ar_fit_begin / npfn_ar_fit_step under a fit token
    (every step's preprocessing queued on the side stream at once), and a second pass of the
    loop under the same token reuses those fits; otherwise npfn_fit per step."""
    from npe_pfn.distributed import canonical_order
    from npe_pfn.engine import Engine

    theta, x, x_o = gaussian_linear_task(4, 300, seed=1)
    N = 777  # unequal row shards
    xq = (x_o.repeat(N, 1) + 0.02 * torch.randn(N, 4, generator=torch.Generator().manual_seed(2))).to(DEV)
    ref = Engine(CFG, weights, device=DEV, random_state=4)
    ref.set_preprocessing(pre)
    th_ref, lp_ref = ref.ar_sample(x, theta, xq, counter=5, with_log_prob=True)
    del ref
    E = CFG.n_estimators
    engs = []
    for r in range(G):
        e = Engine(CFG, weights, device=DEV, random_state=4)
        e.set_preprocessing(pre)
        if strided:
            e.set_estimator_set(r, E // G, G)
        else:
            e.set_estimator_range(r * E // G, E // G)
        engs.append(e)
    joint = torch.cat([x, theta], 1).to(DEV)
    bounds = [shard_bounds(N, r, G) for r in range(G)]
    if stepwise:
        for e in engs:
            e.set_fit_token(77)
    for _ in range(2 if stepwise else 1):
        feat = xq.clone()
        lps = [torch.zeros(b - a, device=DEV) for a, b in bounds]
        if stepwise:
            for e in engs:
                e.ar_fit_begin(x, theta)
        for k in range(theta.shape[1]):
            toks = []
            for e in engs:
                if stepwise:
                    e.ar_fit_step(k)
                else:
                    e.fit(joint[:, : 4 + k], joint[:, 4 + k])
                toks.append(e.forward_targets(feat))
            full = torch.cat(toks, 0)  # rank-major
            if strided:
                full = canonical_order(full, G)
            assert full.shape == (E, N, CFG.d_model)
            col = torch.cat([engs[r].head_sample(full[:, a:b].contiguous(), 5 + k, row_base=a, log_prob_acc=lps[r])
                             for r, (a, b) in enumerate(bounds)])
            feat = torch.cat([feat, col[:, None]], 1)
        assert torch.equal(feat[:, 4:], th_ref), (feat[:, 4:] - th_ref).abs().max()
        assert torch.equal(torch.cat(lps), lp_ref)


def test_partial_range_refuses_mixing_calls(weights):
    """The C engine refuses the ensemble-mixing calls under a partial estimator range; the
    Python Engine's ar_sample / ar_log_prob restore the full range first (after an
    estimator-parallel call the posterior's other entry points keep working)."""
    import ctypes

    from npe_pfn.engine import Engine, EngineError

    e = Engine(CFG, weights, device=DEV, random_state=0, preprocessing="none")
    e.set_estimator_range(2, 3)
    theta, x, x_o = gaussian_linear_task(2, 50, seed=0)
    xd, thd, xq = x.to(DEV).contiguous(), theta.to(DEV).contiguous(), x_o.repeat(4, 1).to(DEV).contiguous()
    out = torch.empty((4, 2), device=DEV)
    rc = e.lib.npfn_ar_sample(e.h, ctypes.c_void_p(xd.data_ptr()), ctypes.c_void_p(thd.data_ptr()), 50, 2, 2,
                              ctypes.c_void_p(xq.data_ptr()), 4, 0, 0, ctypes.c_void_p(out.data_ptr()), None,
                              1e-15, e.stream)
    assert rc != 0 and b"estimator_range" in e.lib.npfn_last_error()
    e.fit(x, theta[:, 0])
    assert e.forward_targets(x_o.repeat(4, 1)).shape == (3, 4, CFG.d_model)
    with pytest.raises(EngineError, match="estimator_range"):
        e.predict_logits(x_o.repeat(4, 1))
    th, _ = e.ar_sample(x, theta, x_o.repeat(4, 1), counter=0)  # restores (0, E)
    assert (e.e0, e.ne) == (0, CFG.n_estimators) and torch.isfinite(th).all()


def test_ep_sample_then_plain_log_prob():
    """An estimator-parallel sample leaves the posterior usable: log_prob / sample on the same
    posterior afterwards (the EP call restores the full estimator range)."""
    from npe_pfn import TabPFN_Based_NPE_PFN
    from npe_pfn.distributed import sample_estimator_parallel

    theta, x, x_o = gaussian_linear_task(3, 300, seed=2)
    post = TabPFN_Based_NPE_PFN(prior=gaussian_linear_prior(3, device=DEV),
                                regressor_init_kwargs={"random_state": 1, "device": DEV})
    post.append_simulations(theta.to(DEV), x.to(DEV))
    s = sample_estimator_parallel(post, x_o.to(DEV), (500,))
    lp = post.log_prob(s[:50], x_o.to(DEV))
    assert torch.isfinite(lp).all()
    assert post.sample((100,), x=x_o.to(DEV)).shape == (100, 3)


def test_sample_estimator_parallel_single_rank_equals_sample():
    """The public estimator-parallel sample (world 1: one rank holds every estimator and the
    loop runs through forward_targets + head_sample) == the fused TabPFN_Based_NPE_PFN.sample."""
    from npe_pfn import TabPFN_Based_NPE_PFN
    from npe_pfn.distributed import sample_estimator_parallel

    theta, x, x_o = gaussian_linear_task(5, 400, seed=3)
    out = []
    for ep in (False, True):
        post = TabPFN_Based_NPE_PFN(prior=gaussian_linear_prior(5, device=DEV),
                                    regressor_init_kwargs={"random_state": 6, "device": DEV})
        post.append_simulations(theta.to(DEV), x.to(DEV))
        if ep:
            out.append(sample_estimator_parallel(post, x_o.to(DEV), (2000,), with_log_prob=True))
        else:
            out.append(post.sample((2000,), x=x_o.to(DEV), with_log_prob=True))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
