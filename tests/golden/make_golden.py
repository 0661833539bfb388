"""Generate golden vectors by running the REFERENCE orchestration with the oracle plugged in.

Run here (never on the GPU box -- /root/reference does not exist there):

    python tests/golden/make_golden.py

What it does
------------
The reference's hot-path Python (``npe_pfn/npe_pfn.py``,
``npe_pfn/accept_reject_sampler.py``, ``npe_pfn/support_posterior.py``) is
loaded BY PATH from /root/reference, with two in-process stand-ins for the
absent third-party imports:

* ``tabpfn.TabPFNRegressor`` -> ``oracle.tabpfn_oracle.OracleRegressor`` and
  ``tabpfn.TabPFNClassifier`` -> ``oracle.tabpfn_oracle.OracleClassifier`` (the
  CPU restatement; the classifier runs on the synthetic classifier weights);
* ``sbi.utils.BoxUniform`` -> a torch ``Independent(Uniform)`` with the same
  constructor (sbi 0.23.3, poetry.lock:4225).

The reference then drives the oracle through its own call sequence, and the
inputs, outputs and the recorded fit/predict call log are saved as ``.npz``
fixtures.  Nothing from the reference is copied into the fixtures except data
(inputs / outputs / shapes).
"""

from __future__ import annotations

import importlib
import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference/npe_pfn"
sys.path.insert(0, REPO)

from oracle.tabpfn_oracle import OracleClassifier, OracleRegressor  # noqa: E402


def _load_weights_module():
    spec = importlib.util.spec_from_file_location(
        "npfn_weights_for_golden", os.path.join(REPO, "npe-pfn_amd", "npe_pfn", "weights.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod
    spec.loader.exec_module(mod)
    return mod


def install_reference():
    """Load the reference modules by path under their own package name."""
    tabpfn = types.ModuleType("tabpfn")
    tabpfn.TabPFNRegressor = OracleRegressor
    tabpfn.TabPFNClassifier = OracleClassifier
    sys.modules["tabpfn"] = tabpfn

    sbi = types.ModuleType("sbi")
    sbi_utils = types.ModuleType("sbi.utils")

    class BoxUniform(torch.distributions.Independent):
        def __init__(self, low, high, reinterpreted_batch_ndims=1, device=None):
            super().__init__(torch.distributions.Uniform(torch.as_tensor(low, dtype=torch.float32),
                                                         torch.as_tensor(high, dtype=torch.float32)),
                             reinterpreted_batch_ndims)

    sbi_utils.BoxUniform = BoxUniform
    sbi.utils = sbi_utils
    sys.modules["sbi"] = sbi
    sys.modules["sbi.utils"] = sbi_utils

    pkg = types.ModuleType("npe_pfn")
    pkg.__path__ = [REF]
    sys.modules["npe_pfn"] = pkg
    mods = {}
    for name in ("accept_reject_sampler", "support_posterior", "npe_pfn"):
        mods[name] = importlib.import_module(f"npe_pfn.{name}")
    return mods, BoxUniform


def gl_task(D: int, n_sims: int, seed: int):
    """Gaussian-linear (sbibm): theta ~ N(0, 0.1 I), x = theta + sqrt(0.1) eps."""
    g = torch.Generator().manual_seed(seed)
    theta = torch.randn(n_sims, D, generator=g) * np.sqrt(0.1)
    x = theta + torch.randn(n_sims, D, generator=g) * np.sqrt(0.1)
    g2 = torch.Generator().manual_seed(seed + 1)
    theta_o = torch.randn(1, D, generator=g2) * np.sqrt(0.1)
    x_o = theta_o + torch.randn(1, D, generator=g2) * np.sqrt(0.1)
    return theta.float(), x.float(), x_o.float()


def main():
    W = _load_weights_module()
    cfg = W.ModelConfig()
    weights = W.synthetic_weights(cfg, seed=0)
    OracleRegressor.default_weights = weights
    digest = W.weights_digest(weights, cfg)
    ccfg = W.classifier_config()
    cweights = W.synthetic_classifier_weights(ccfg, seed=1)
    OracleClassifier.default_weights = cweights
    cdigest = W.weights_digest(cweights, ccfg)
    mods, BoxUniform = install_reference()
    ref = mods["npe_pfn"]
    out = {}

    # ---- case c1: GL-2D, 200 sims, 1000 samples, NPE_PFN_Core, Gaussian prior
    theta, x, x_o = gl_task(2, 200, seed=0)
    prior = torch.distributions.Independent(
        torch.distributions.Normal(torch.zeros(2), torch.full((2,), float(np.sqrt(0.1)))), 1)
    core = ref.NPE_PFN_Core(prior=prior, regressor_init_kwargs={"random_state": 7})
    core.append_simulations(theta, x)
    s, lp = core.sample((1000,), x=x_o, with_log_prob=True)
    lp_ar = core.log_prob(s[:200], x_o)
    out["c1"] = dict(theta=theta.numpy(), x=x.numpy(), x_o=x_o.numpy(), samples=s.numpy(),
                     log_probs=lp.numpy(), log_prob_ar=lp_ar.numpy(),
                     calls=json.dumps(core._model.calls), random_state=7)

    # ---- case filt: TabPFN_Based_NPE_PFN, std-euclid filter to 64 of 200 sims
    theta, x, x_o = gl_task(3, 200, seed=3)
    prior3 = torch.distributions.Independent(
        torch.distributions.Normal(torch.zeros(3), torch.full((3,), float(np.sqrt(0.1)))), 1)
    post = ref.TabPFN_Based_NPE_PFN(prior=prior3, filter_type="standardized_euclidean_filtering",
                                    filter_context_size=64, regressor_init_kwargs={"random_state": 11})
    post.append_simulations(theta, x)
    s, lp = post.sample((200,), x=x_o, with_log_prob=True)
    out["filt"] = dict(theta=theta.numpy(), x=x.numpy(), x_o=x_o.numpy(), samples=s.numpy(),
                       log_probs=lp.numpy(), calls=json.dumps(post._model.calls), random_state=11)

    # ---- case box: BoxUniform prior, rejection loop with batch-size recurrence
    g = torch.Generator().manual_seed(5)
    theta = (torch.rand(150, 2, generator=g) * 2 - 1) * 1.0
    x = theta + 0.3 * torch.randn(150, 2, generator=g)
    x_o = torch.tensor([[0.8, -0.7]])
    box = BoxUniform(torch.full((2,), -0.95), torch.full((2,), 0.95))
    core = ref.NPE_PFN_Core(prior=box, regressor_init_kwargs={"random_state": 3})
    core.append_simulations(theta, x)
    s = core.sample((300,), x=x_o, max_sampling_batch_size=250)
    out["box"] = dict(theta=theta.numpy(), x=x.numpy(), x_o=x_o.numpy(), samples=s.numpy(),
                      calls=json.dumps(core._model.calls), random_state=3,
                      low=np.full(2, -0.95, np.float32), high=np.full(2, 0.95, np.float32))

    # ---- case batched: sample_batched, 3 observations x 40 samples, box prior
    g = torch.Generator().manual_seed(9)
    theta = (torch.rand(120, 2, generator=g) * 2 - 1)
    x = theta + 0.2 * torch.randn(120, 2, generator=g)
    xs = torch.tensor([[0.1, 0.2], [-0.5, 0.4], [0.9, 0.9]])
    core = ref.NPE_PFN_Core(prior=BoxUniform(torch.full((2,), -1.0), torch.full((2,), 1.0)),
                            regressor_init_kwargs={"random_state": 5})
    core.append_simulations(theta, x)
    s, lp = core.sample_batched(xs, (40,), with_log_prob=True)
    out["batched"] = dict(theta=theta.numpy(), x=x.numpy(), x_o=xs.numpy(), samples=s.numpy(),
                          log_probs=lp.numpy(), calls=json.dumps(core._model.calls), random_state=5)

    # ---- filters, seeded (random_filtering consumes the global torch RNG)
    sp = mods["support_posterior"]
    g = torch.Generator().manual_seed(21)
    th = torch.randn(500, 3, generator=g)
    xx = torch.randn(500, 4, generator=g) * torch.tensor([1.0, 2.0, 0.5, 3.0])
    ob = torch.randn(1, 4, generator=g)
    filt = {}
    for name in ("no_filtering", "latest_filtering", "random_filtering", "standardized_euclidean_filtering"):
        torch.manual_seed(1234)
        t_c, x_c = sp.get_filtering_method(name)(ob, th, xx, 100)
        filt[name + "_theta"] = t_c.numpy()
        filt[name + "_x"] = x_c.numpy()
    out["filters"] = dict(theta=th.numpy(), x=xx.numpy(), obs=ob.numpy(), **filt)

    # ---- accept/reject recurrence with a deterministic proposal
    ars = mods["accept_reject_sampler"]
    state = {"i": 0}

    def proposal(bs, **kw):
        state["i"] += 1
        gg = torch.Generator().manual_seed(100 + state["i"])
        c = torch.rand(bs, 2, generator=gg)
        return c, c.sum(1)

    trace = []

    def acc(c):
        trace.append(c.shape[0])
        return c[:, 0] < 0.3

    smp, lps, rate = ars.accept_reject_sample(proposal, acc, num_samples=700, max_sampling_batch_size=1000)
    out["accrej"] = dict(samples=smp.numpy(), log_probs=lps.numpy(), rate=np.float64(rate),
                         batch_trace=np.asarray(trace, dtype=np.int64))

    # ---- case ratio: ratio-based log_prob (DensityRatioWrapper + classifier), GL-2D
    theta, x, x_o = gl_task(2, 100, seed=13)
    prior = torch.distributions.Independent(
        torch.distributions.Normal(torch.zeros(2), torch.full((2,), float(np.sqrt(0.1)))), 1)
    core = ref.NPE_PFN_Core(prior=prior, regressor_init_kwargs={"random_state": 2},
                            classifier_init_kwargs={"random_state": 4})
    core.append_simulations(theta, x)
    gq = torch.Generator().manual_seed(17)
    th_q = torch.randn(40, 2, generator=gq) * 0.6
    torch.manual_seed(4321)
    lp_ratio = core.log_prob(th_q, x_o, mode="ratio_based", num_posterior_samples=100)
    lp_ratio2 = core.log_prob(th_q[:10], x_o, mode="ratio_based", num_posterior_samples=100)  # reuses the fit
    wrap = core._model_classifier
    out["ratio"] = dict(theta=theta.numpy(), x=x.numpy(), x_o=x_o.numpy(), theta_q=th_q.numpy(),
                        log_prob=lp_ratio.numpy(), log_prob_reuse=lp_ratio2.numpy(),
                        pad_min=wrap._padded_dim_min.numpy(), pad_max=wrap._padded_dim_max.numpy(),
                        clf_calls=json.dumps(wrap._classifier.calls), reg_calls=json.dumps(core._model.calls),
                        random_state=2, clf_random_state=4, torch_seed=4321)

    meta = dict(weights_seed=0, weights_digest=digest, config=cfg.to_dict(),
                classifier_weights_seed=1, classifier_weights_digest=cdigest, classifier_config=ccfg.to_dict(),
                generator="tests/golden/make_golden.py", reference="/root/reference @ 2026-02-06")
    for case, arrays in out.items():
        np.savez(os.path.join(HERE, f"{case}.npz"), **arrays)
    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", sorted(out), "digest", digest)


if __name__ == "__main__":
    main()
