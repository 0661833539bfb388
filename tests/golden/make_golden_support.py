"""Golden vectors for PosteriorSupport (rejection and SIR) from the REFERENCE's own code.

Run here (never on the GPU box -- /root/reference does not exist there):

    python tests/golden/make_golden_support.py

Loads the reference's support_posterior.py / npe_pfn.py by path exactly as
make_golden.py does (oracle as ``tabpfn``), builds a TabPFN_Based_NPE_PFN on a
small GL-2D context and records what PosteriorSupport returns for both sampling
methods under fixed torch seeds (the reference's draws of prior samples and of
the SIR Categorical come from torch's global RNG; the oracle's bar sampling from
Philox).  Writes tests/golden/support.npz (data only).
"""

from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import REPO, _load_weights_module, gl_task, install_reference  # noqa: E402

sys.path.insert(0, REPO)
from oracle.tabpfn_oracle import OracleRegressor  # noqa: E402


def main():
    W = _load_weights_module()
    OracleRegressor.default_weights = W.synthetic_weights(W.ModelConfig(), seed=0)
    mods, _ = install_reference()
    ref, sp = mods["npe_pfn"], mods["support_posterior"]
    theta, x, x_o = gl_task(2, 100, seed=31)
    prior = torch.distributions.Independent(
        torch.distributions.Normal(torch.zeros(2), torch.full((2,), float(np.sqrt(0.1)))), 1)
    out = dict(theta=theta.numpy(), x=x.numpy(), x_o=x_o.numpy(), random_state=np.int64(6))

    post = ref.TabPFN_Based_NPE_PFN(prior=prior, regressor_init_kwargs={"random_state": 6})
    post.append_simulations(theta, x)
    torch.manual_seed(2024)
    sup = sp.PosteriorSupport(prior, post, x_o, num_samples_to_estimate_support=200,
                              batch_size_for_estimate_support=200, allowed_false_negatives=0.05,
                              sampling_method="rejection")
    s, rate = sup.sample((150,), show_progress_bars=False, sampling_batch_size=100, return_acceptance_rate=True)
    out.update(rej_thr=np.float32(sup.thr), rej_samples=s.numpy(), rej_rate=np.float64(rate),
               rej_calls=json.dumps(post._model.calls))

    post = ref.TabPFN_Based_NPE_PFN(prior=prior, regressor_init_kwargs={"random_state": 6})
    post.append_simulations(theta, x)
    torch.manual_seed(77)
    sup = sp.PosteriorSupport(prior, post, x_o, allowed_false_negatives=0.05, sampling_method="sir",
                              oversample_sir=10)
    s, ess = sup.sample((25,), show_progress_bars=False, sampling_batch_size=100, return_ess=True)
    out.update(sir_samples=s.numpy(), sir_ess=ess.numpy(), sir_calls=json.dumps(post._model.calls))
    np.savez(os.path.join(HERE, "support.npz"), **out)
    print("wrote support.npz", {k: getattr(v, "shape", None) for k, v in out.items()})


if __name__ == "__main__":
    main()
