"""Golden vectors for config c4 (the demo's TSNPE-PFN recipe) from the REFERENCE.

Run here (never on the GPU box -- /root/reference does not exist there):

    python tests/golden/make_golden_c4.py [num_samples_to_estimate_support]

Loads the reference's tsnpe_pfn.py, npe_pfn.py, support_posterior.py and accept_reject_sampler.py
by path with the CPU oracle as ``tabpfn`` (OracleRegressor / OracleClassifier at the FULL
architecture: the synthetic TabPFN-v2 regressor weights seed 0 and classifier weights seed 1, the
engine's defaults, and the default preprocessing ensembles) and with sbi's ``simulate_for_sbi``
restated on the reference's call path (as make_golden_tsnpe.py), then runs the demo's recipe
(/root/reference/demo.ipynb:357-364): the two-moons simulator (demo.ipynb:50-75) under the plain
``Uniform(-1, 1)`` prior (:78), x_o simulated at theta_o = 0.5 * 1 (:89) after
``torch.manual_seed(42)``, then ``run_tsnpe_pfn(num_simulations=1000, num_rounds=5,
proposal_batch_size=1000, simulation_batch_size=1000)`` with every other argument at the
reference's default -- ``log_prob_mode="ratio_based"``, ``sampling_method="rejection"``,
``num_samples_to_estimate_support=10_000``, ``allowed_false_negatives=1e-4`` -- after
``torch.manual_seed(0)``; finally 1000 draws of the final posterior at x_o (demo.ipynb, the cell
after the run).  An optional argument reduces ``num_samples_to_estimate_support`` (only if the
full recipe does not finish in the container; the fixture records the value used).

Writes tests/golden/c4.npz (data only): x_o, every round's (theta, x), the final draws, and the
recipe's parameters, for tests/test_gpu_c4_posterior.py.
"""

from __future__ import annotations

import importlib
import logging
import os
import sys
import time
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import REF, REPO, _load_weights_module, install_reference  # noqa: E402
from make_golden_tsnpe import simulate_for_sbi  # noqa: E402

sys.path.insert(0, REPO)
from oracle.tabpfn_oracle import OracleClassifier, OracleRegressor  # noqa: E402

RECIPE = dict(num_simulations=1000, num_rounds=5, proposal_batch_size=1000, simulation_batch_size=1000)
N_DRAWS = 1000


def two_moons_simulator(theta):
    """demo.ipynb:50-75 (global torch RNG)."""
    n = theta.shape[0]
    a = torch.distributions.Uniform(torch.zeros(n) + (-np.pi / 2), torch.zeros(n) + (np.pi / 2)).rsample()
    r = torch.distributions.Normal(torch.zeros(n) + 0.1, torch.zeros(n) + 0.01).rsample()
    p = torch.empty(theta.shape)
    p[:, 0] = torch.mul(r, torch.cos(a)) + 0.25
    p[:, 1] = torch.mul(r, torch.sin(a))
    q = torch.empty(theta.shape)
    q[:, 0] = -torch.abs(theta[:, 0] + theta[:, 1]) / np.sqrt(2)
    q[:, 1] = (-theta[:, 0] + theta[:, 1]) / np.sqrt(2)
    return p + q


def main():
    support_n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(message)s")
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
    prior = torch.distributions.Uniform(-torch.ones(2), torch.ones(2))
    torch.manual_seed(42)
    x_o = two_moons_simulator(0.5 * torch.ones(1, 2))
    torch.manual_seed(0)
    t0 = time.time()
    post = tsnpe.run_tsnpe_pfn(two_moons_simulator, prior, x_o, num_samples_to_estimate_support=support_n, **RECIPE)
    print(f"reference c4 run_tsnpe_pfn: {time.time() - t0:.1f} s", flush=True)
    torch.manual_seed(1)
    s = post.sample((N_DRAWS,), x=x_o)
    print(f"reference c4 final draws: {time.time() - t0:.1f} s, {tuple(s.shape)}", flush=True)
    np.savez(os.path.join(HERE, "c4.npz"), x_o=x_o.numpy(), theta=post._theta_train.numpy(),
             x=post._x_train.numpy(), samples=s.numpy(), num_samples_to_estimate_support=support_n,
             num_simulations=RECIPE["num_simulations"], num_rounds=RECIPE["num_rounds"],
             proposal_batch_size=RECIPE["proposal_batch_size"])


if __name__ == "__main__":
    main()
