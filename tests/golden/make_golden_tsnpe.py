"""Golden vectors for the TSNPE-PFN round loop (config c4's orchestration) from the REFERENCE.

Run here (never on the GPU box -- /root/reference does not exist there):

    python tests/golden/make_golden_tsnpe.py

Loads the reference's tsnpe_pfn.py, npe_pfn.py, support_posterior.py and
accept_reject_sampler.py by path (oracle as ``tabpfn``, as make_golden.py), with one more
stand-in: ``sbi.inference.simulate_for_sbi`` (sbi 0.23.3, poetry.lock:4225; absent here),
restated from its published code path with the defaults the reference uses
(tsnpe_pfn.py:86-91: num_workers=1, seed=None): ``theta = proposal.sample((n,))`` then the
simulator on ``torch.split(theta, simulation_batch_size)`` in order, outputs concatenated.
The reference loop then runs, with a 1-layer / 64-bar synthetic estimator of the same
architecture (cheap: the fixture pins the round loop, not the forward), 3 rounds x 40 simulations of a Gaussian-linear 2D simulator
under a box prior, with the autoregressive log density for the support threshold and SIR
proposals (the ratio-based density needs a 10 000-row classifier context and the rejection
proposal 10 000-row prior batches: out of reach of the CPU oracle in a test; their
orchestration is pinned by ratio.npz and support.npz).  Writes tests/golden/tsnpe.npz
(data only): every round's (theta, x) and 300 posterior draws of the final estimator.
"""

from __future__ import annotations

import importlib
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import REF, REPO, _load_weights_module, install_reference  # noqa: E402

sys.path.insert(0, REPO)
from oracle.tabpfn_oracle import OracleClassifier, OracleRegressor  # noqa: E402

TSNPE_KW = dict(num_simulations=120, num_rounds=3, proposal_batch_size=100, simulation_batch_size=16,
                num_samples_to_estimate_support=200, allowed_false_negatives=0.05,
                log_prob_mode="autoregressive", sampling_method="sir", oversample_sir=10)
# a small estimator of the same architecture (1 layer, 64 bars): the golden pins the round
# loop, the simulations and the proposals, not the forward, so it only has to be cheap
TINY = dict(n_layers=1, d_ff=192, n_bars=64, max_groups=16)


def regressor_kwargs(W):
    return {"random_state": 9, "preprocessing": "none", "weights": W.synthetic_weights(W.ModelConfig(**TINY), seed=3)}


def simulate_for_sbi(simulator, proposal, num_simulations, num_workers=1, simulation_batch_size=1, seed=None,
                     show_progress_bar=True):
    """sbi 0.23.3 ``simulate_for_sbi`` on the reference's call path (num_workers=1, seed=None)."""
    theta = proposal.sample((num_simulations,))
    xs = [simulator(b) for b in torch.split(theta, simulation_batch_size, dim=0)]
    return theta, torch.cat(xs, dim=0)


def simulator(theta):
    """Gaussian-linear 2D with the global torch RNG (as the demo's two-moons simulator)."""
    return theta + 0.3 * torch.randn(theta.shape)


def main():
    W = _load_weights_module()
    OracleRegressor.default_weights = W.synthetic_weights(W.ModelConfig(), seed=0)
    OracleClassifier.default_weights = W.synthetic_classifier_weights(W.classifier_config(), seed=1)
    install_reference()
    inf = types.ModuleType("sbi.inference")
    inf.simulate_for_sbi = simulate_for_sbi
    sys.modules["sbi.inference"] = inf
    sys.modules["sbi"].inference = inf
    tsnpe = importlib.import_module("npe_pfn.tsnpe_pfn")
    assert os.path.dirname(tsnpe.__file__) == REF
    BoxUniform = sys.modules["sbi.utils"].BoxUniform
    prior = BoxUniform(torch.full((2,), -1.5), torch.full((2,), 1.5))
    x_o = torch.tensor([[0.4, -0.3]])
    torch.manual_seed(123)
    post = tsnpe.run_tsnpe_pfn(simulator, prior, x_o, regressor_init_kwargs=regressor_kwargs(W), **TSNPE_KW)
    th, x = post._theta_train, post._x_train
    torch.manual_seed(321)
    s = post.sample((300,), x=x_o)
    np.savez(os.path.join(HERE, "tsnpe.npz"), theta=th.numpy(), x=x.numpy(), x_o=x_o.numpy(), samples=s.numpy(),
             low=np.float32(-1.5), high=np.float32(1.5))
    print("wrote tsnpe.npz", th.shape, s.shape)


if __name__ == "__main__":
    main()
