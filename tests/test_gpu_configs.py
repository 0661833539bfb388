"""Every BASELINE.json config through the HIP path.

* c2 parity (GL-10D, 1000 simulations): the engine's predictive bar distribution at the
  first (F = 10 features, C = 6 tokens), a middle (F = 14, C = 8) and the last
  (F = 19, C = 11) autoregressive step against the bf16-emulating oracle on a 256-row
  query subset.  Tolerance as tests/test_gpu_engine.py: total variation per row <= 0.02
  (bf16 oracle), <= 0.05 (fp32 oracle).  These C values run the row kernel's 42 / 32 / 23
  rows-per-tile packings (npfn_rowk2.hip rowk_rows_per_tile, 256 token slots).
* c2 / c3 / c4 / c5 at full size: the public calls (``TabPFN_Based_NPE_PFN.sample``,
  ``run_tsnpe_pfn``, ``sample_batched``) with shape, finiteness and prior-support
  properties -- posterior quality is not testable on synthetic weights.
* chunk boundaries: ``npfn_set_chunk_rows`` splits one predict into many chunks; the
  draws equal the single-chunk draws bit for bit (the forward is batch-invariant: a row's
  feature attention does not depend on its slot in the row tile), and a shard whose
  ``row_base`` starts inside chunk 2 draws the unsharded rows' numbers.
"""
import numpy as np
import pytest
import torch

from npe_pfn.tasks import gaussian_linear_prior, gaussian_linear_task, slcp_prior, slcp_task
from npe_pfn.weights import ModelConfig, synthetic_weights
from oracle.tabpfn_oracle import OracleTabPFN

pytestmark = pytest.mark.gpu

CFG = ModelConfig()
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def weights():
    return synthetic_weights(CFG, seed=0)


@pytest.fixture(scope="module")
def c2_task():
    return gaussian_linear_task(10, 1000, seed=0)


@pytest.mark.parametrize("k,mode", [(0, "none"), (4, "none"), (9, "none"), (0, "ensemble"), (9, "ensemble")])
def test_c2_predict_matches_oracle(weights, c2_task, k, mode):
    """Step k of the c2 AR loop: fit on [x, theta_<k] -> theta_k, predict 256 query rows; with
    the default ensemble preprocessing the estimators run C = 14 / 25 (quantile + SVD +
    fingerprint) and 7 / 11 (Yeo-Johnson + fingerprint) tokens."""
    from npe_pfn.engine import Engine
    from oracle.preprocess_oracle import MODE_ENSEMBLE

    theta, x, x_o = (t.numpy() for t in c2_task)
    X = np.concatenate([x, theta[:, :k]], 1)
    y = theta[:, k]
    rng = np.random.default_rng(k)
    Xq = np.concatenate([np.repeat(x_o, 256, 0), theta[rng.integers(0, 1000, 256), :k]], 1).astype(np.float32)
    eng = Engine(CFG, weights, device=DEV, random_state=2)
    eng.set_preprocessing(mode)
    eng.fit(torch.from_numpy(X), torch.from_numpy(y))
    p_gpu = torch.softmax(eng.predict_logits(torch.from_numpy(Xq)), -1).double().cpu().numpy()
    assert np.isfinite(p_gpu).all()
    modes = ((True, 0.02), (False, 0.05)) if (k == 9 and mode == "none") else ((True, 0.02),)
    for emulate, tol in modes:
        orc = OracleTabPFN(weights, CFG.n_estimators, CFG.softmax_temperature, seed=2, emulate_bf16=emulate,
                           preprocessing=MODE_ENSEMBLE if mode == "ensemble" else 0)
        orc.fit(X, y)
        tv = 0.5 * np.abs(p_gpu - orc.predict_probs(Xq).astype(np.float64)).sum(1)
        print(f"c2 step {k} (F={X.shape[1]}): TV max {tv.max():.4f} mean {tv.mean():.4f} (bf16 oracle={emulate})")
        assert tv.max() <= tol, (k, emulate, tv.max(), tv.mean())


def _c2_posterior(random_state=0, preprocessing="ensemble"):
    from npe_pfn import TabPFN_Based_NPE_PFN

    theta, x, x_o = gaussian_linear_task(10, 1000, seed=0)
    post = TabPFN_Based_NPE_PFN(prior=gaussian_linear_prior(10, device=DEV),
                                regressor_init_kwargs={"random_state": random_state, "device": DEV,
                                                       "preprocessing": preprocessing})
    post.append_simulations(theta.to(DEV), x.to(DEV))
    return post, theta, x_o.to(DEV)


def test_c2_full_sample_properties_and_determinism():
    """c2 at its size: 10 000 draws x 10 dims; a fresh estimator repeats them bit for bit."""
    post, theta, x_o = _c2_posterior()
    s, lp = post.sample((10_000,), x=x_o, with_log_prob=True)
    assert s.shape == (10_000, 10) and lp.shape == (10_000,)
    assert torch.isfinite(s).all() and torch.isfinite(lp).all()
    # every draw lies inside the bar support of its step (borders * std + mean; the half-normal
    # tails of the end bars are not sampled by the inverse CDF)
    lo = theta.min(0).values.to(DEV) - 20 * theta.std(0).to(DEV)
    hi = theta.max(0).values.to(DEV) + 20 * theta.std(0).to(DEV)
    assert ((s >= lo) & (s <= hi)).all()
    assert (s.std(0) > 1e-3).all()               # not collapsed onto one bar
    post2, _, _ = _c2_posterior()
    s2, lp2 = post2.sample((10_000,), x=x_o, with_log_prob=True)
    assert torch.equal(s, s2) and torch.equal(lp, lp2)


def test_c3_slcp_full_sample_in_support():
    """c3: SLCP, 1000 simulations, 10 000 draws with box-prior rejection U(-3, 3)^5."""
    from npe_pfn import TabPFN_Based_NPE_PFN

    theta, x, x_o = slcp_task(1000, seed=0)
    post = TabPFN_Based_NPE_PFN(prior=slcp_prior(device=DEV), regressor_init_kwargs={"random_state": 0, "device": DEV})
    post.append_simulations(theta.to(DEV), x.to(DEV))
    s = post.sample((10_000,), x=x_o.to(DEV))
    assert s.shape == (10_000, 5) and torch.isfinite(s).all()
    assert ((s >= -3) & (s <= 3)).all()
    assert (s.std(0) > 1e-3).all()


def test_c4_tsnpe_two_moons_full_size():
    """c4: TSNPE-PFN, 5 rounds x 200 simulations, proposal_batch_size 1000 (demo.ipynb:357-364),
    ratio-based support estimate with 10 000 posterior samples per round (the defaults)."""
    from npe_pfn import run_tsnpe_pfn
    from npe_pfn.tasks import two_moons_prior, two_moons_simulator

    torch.manual_seed(0)
    prior = two_moons_prior()
    x_o = two_moons_simulator(0.5 * torch.ones(1, 2))
    post = run_tsnpe_pfn(two_moons_simulator, prior, x_o, num_simulations=1000, num_rounds=5,
                         proposal_batch_size=1000, regressor_init_kwargs={"device": DEV},
                         classifier_init_kwargs={"device": DEV})
    assert post._theta_train.shape == (1000, 2)
    s = post.sample((10_000,), x=x_o)
    assert s.shape == (10_000, 2) and torch.isfinite(s).all()
    assert ((s >= -1) & (s <= 1)).all()


def test_c5_64_obs_full_size():
    """c5: 64 observations x 10 000 draws through sample_batched (960 000 query rows per step,
    59 predict chunks per AR step at the default chunk size)."""
    from npe_pfn import NPE_PFN_Core

    theta, x, _ = gaussian_linear_task(10, 1000, seed=0)
    x_obs = gaussian_linear_task(10, 64, seed=123)[1].to(DEV)
    post = NPE_PFN_Core(prior=gaussian_linear_prior(10, device=DEV),
                        regressor_init_kwargs={"random_state": 0, "device": DEV})
    post.append_simulations(theta.to(DEV), x.to(DEV))
    s, lp = post.sample_batched(x_obs, (10_000,), with_log_prob=True)
    assert s.shape == (64, 10_000, 10) and lp.shape == (64, 10_000)
    assert torch.isfinite(s).all() and torch.isfinite(lp).all()
    # observations differ, so their posteriors do
    assert (s[:, :, 0].mean(1).std() > 0)


def test_chunk_boundaries_and_row_base_inside_chunk2(weights):
    """npfn_set_chunk_rows: 700 query rows in chunks of 128 vs one chunk; a shard of rows
    [300, 700) (inside chunk 2 onwards) with row_base 300 draws the same numbers -- bit for bit:
    the forward is batch-invariant (a row's result does not depend on its slot in the row
    kernel's tile, npfn_rowk2.hip feat_attn_rows), as the reference's one predict over all rows
    (npe_pfn.py:217) is."""
    from npe_pfn.engine import Engine

    theta, x, x_o = gaussian_linear_task(4, 400, seed=3)
    rng = np.random.default_rng(0)
    xq = torch.from_numpy((np.repeat(x_o.numpy(), 700, 0) + 0.05 * rng.normal(size=(700, 4))).astype(np.float32))
    eng = Engine(CFG, weights, device=DEV, random_state=5, preprocessing="none")
    ref, lp_ref = eng.ar_sample(x, theta, xq, counter=3, with_log_prob=True)
    eng.set_chunk_rows(128)
    ch, lp_ch = eng.ar_sample(x, theta, xq, counter=3, with_log_prob=True)
    sh, lp_sh = eng.ar_sample(x, theta, xq[300:], counter=3, with_log_prob=True, row_base=300)
    for got, lp in ((ch, lp_ch), (torch.cat([ch[:300], sh]), torch.cat([lp_ch[:300], lp_sh]))):
        assert torch.equal(got, ref), (got - ref).abs().max()
        assert torch.equal(lp, lp_ref), (lp - lp_ref).abs().max()
    # the identical call is bitwise reproducible
    ch2, _ = eng.ar_sample(x, theta, xq, counter=3, with_log_prob=True)
    assert torch.equal(ch, ch2)


@pytest.mark.parametrize("mode", ["none", "quantile", "quantile+power", "ensemble"])
def test_logits_bitwise_identical_across_engines(weights, mode):
    """Determinism: three engines, same inputs -> bitwise-identical logits (every
    reduction has a fixed order; k_power_fit's compaction no longer depends on thread
    arrival, c3c8c31)."""
    from npe_pfn.engine import Engine

    rng = np.random.default_rng(0)
    X = torch.from_numpy(np.exp(rng.normal(size=(1000, 6))).astype(np.float32))
    y = torch.from_numpy(rng.normal(size=1000).astype(np.float32))
    Xq = torch.from_numpy(np.exp(rng.normal(size=(500, 6))).astype(np.float32))
    outs = []
    for _ in range(3):
        e = Engine(CFG, weights, device=DEV, random_state=1)
        e.set_preprocessing(mode)
        e.fit(X, y)
        outs.append(e.predict_logits(Xq).cpu())
        del e
    assert all(torch.equal(outs[0], o) for o in outs[1:])


def test_ar_sample_bitwise_identical_at_c2_shape(weights, c2_task):
    """Determinism of the fused sampler at c2's shape (1000 context rows, 10 000 queries,
    10 AR dims): two engines draw identical samples and log-probs."""
    from npe_pfn.engine import Engine

    theta, x, x_o = c2_task
    xq = x_o.repeat(10_000, 1)
    res = []
    for _ in range(2):
        e = Engine(CFG, weights, device=DEV, random_state=0, preprocessing="none")
        res.append(e.ar_sample(x, theta, xq, counter=0, with_log_prob=True))
        del e
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def test_fit_reuse_across_accept_reject_batches():
    """One sample() call fits every AR step once (npfn_set_fit_token), not once per
    accept/reject batch as the reference does (npe_pfn.py:135-140 from accept_reject_sampler.py:51);
    the fit is deterministic, so the draws are bit for bit those of refitting every batch."""
    import contextlib

    from npe_pfn import TabPFN_Based_NPE_PFN

    theta, x, x_o = slcp_task(1000, seed=0)
    out, fits = [], []
    for reuse in (True, False):
        post = TabPFN_Based_NPE_PFN(prior=slcp_prior(device=DEV),
                                    regressor_init_kwargs={"random_state": 3, "device": DEV})
        post.append_simulations(theta.to(DEV), x.to(DEV))
        if not reuse:
            post._model.reuse_fits = contextlib.nullcontext
        eng = post._model.engine
        eng.prof_read()
        eng.prof_enable(True)
        out.append(post.sample((3000,), x=x_o.to(DEV), max_sampling_batch_size=1000))
        eng.prof_enable(False)
        prof = {e["name"]: e["launches"] for e in eng.prof_read()}
        fits.append(prof["k_col_stats+k_build_params"])
    assert torch.equal(out[0], out[1])
    assert fits[0] == 5, fits            # one fit per AR dimension
    assert fits[1] >= 3 * 5, fits        # >= 3 batches, each refitting every dimension


@pytest.mark.parametrize("n_obs,per,pre", [(1, 3000, "ensemble"), (3, 700, "ensemble"), (1, 2000, "none")])
def test_ar_sample_repeated_rows_equal_ar_sample(weights, n_obs, per, pre):
    """npfn_ar_sample_repeated (AR step 0 once per distinct query row, every row drawing from
    its row's mixture) == npfn_ar_sample over the repeated rows, bit for bit (the forward is
    batch-invariant); the same call is bitwise reproducible; a row shard with row_base draws
    the unsharded rows' numbers."""
    from npe_pfn.engine import Engine

    theta, x, _ = gaussian_linear_task(4, 400, seed=4)
    xs = x[:n_obs] + 0.1
    N = n_obs * per
    xq = xs.repeat_interleave(per, 0)
    eng = Engine(CFG, weights, device=DEV, random_state=2)
    eng.set_preprocessing(pre)
    ref, lp_ref = eng.ar_sample(x, theta, xq, counter=4, with_log_prob=True)
    rep, lp_rep = eng.ar_sample(x, theta, xq, counter=4, with_log_prob=True, x_unique=xs)
    assert torch.equal(rep, ref), (rep - ref).abs().max()
    assert torch.equal(lp_rep, lp_ref), (lp_rep - lp_ref).abs().max()
    rep2, lp_rep2 = eng.ar_sample(x, theta, xq, counter=4, with_log_prob=True, x_unique=xs)
    assert torch.equal(rep, rep2) and torch.equal(lp_rep, lp_rep2)
    if n_obs == 1:  # a shard [a, N) of the one-observation batch
        a = N // 3
        sh, lp_sh = eng.ar_sample(x, theta, xq[a:], counter=4, with_log_prob=True, row_base=a, x_unique=xs)
        assert torch.equal(sh, rep[a:]) and torch.equal(lp_sh, lp_rep[a:])
    assert torch.isfinite(rep).all() and torch.isfinite(lp_rep).all()
