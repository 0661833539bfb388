"""Golden vectors for config c5's call (sample_batched over several observations) from the REFERENCE.

Run here (never on the GPU box -- /root/reference does not exist there):

    python tests/golden/make_golden_c5.py

Loads the reference's npe_pfn.py by path with the CPU oracle as ``tabpfn`` (as make_golden.py)
and runs c5's call -- ``NPE_PFN_Core.sample_batched(x_obs, (N,))`` on Gaussian-linear 10D, one
shared context for all observations, the default preprocessing ensemble -- at a size the CPU
oracle finishes in minutes: 300 simulations, 4 observations x 250 samples instead of 1000
simulations, 64 observations x 10 000 samples.  Task data from npe_pfn.tasks
(gaussian_linear_task, seeded; stored in the fixture).  Writes tests/golden/c5.npz (data only).

``python tests/golden/make_golden_c5.py --full`` runs c5's call at its configured context: the
bench's 1 000 simulations (gaussian_linear_task(10, 1000, seed=0)), 8 observations
(gaussian_linear_task(10, 8, seed=123)[1]) x 250 draws through the reference's ``sample_batched``
(1.5x oversampled interleaved batch, per-observation rejection, npe_pfn.py:310-410).  Only the
observation and draw counts are reduced (the oracle's cost).  Writes tests/golden/c5_full.npz,
for tests/test_gpu_c5_posterior.py.
"""

from __future__ import annotations

import importlib.util
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import REPO, _load_weights_module, install_reference  # noqa: E402

sys.path.insert(0, REPO)
from oracle.tabpfn_oracle import OracleRegressor  # noqa: E402

N_SIMS, N_OBS, N_SAMPLES, RANDOM_STATE = 300, 4, 250, 21
FULL_SIMS, FULL_OBS = 1000, 8


def main(full: bool = False):
    W = _load_weights_module()
    OracleRegressor.default_weights = W.synthetic_weights(W.ModelConfig(), seed=0)
    mods, _ = install_reference()
    ref = mods["npe_pfn"]
    spec = importlib.util.spec_from_file_location("npfn_tasks", os.path.join(REPO, "npe-pfn_amd", "npe_pfn", "tasks.py"))
    tasks = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tasks)
    if full:
        theta, x, _ = tasks.gaussian_linear_task(10, FULL_SIMS, seed=0)
        x_obs = tasks.gaussian_linear_task(10, FULL_OBS, seed=123)[1]
    else:
        theta, x, _ = tasks.gaussian_linear_task(10, N_SIMS, seed=6)
        x_obs = tasks.gaussian_linear_task(10, N_OBS, seed=77)[1]
    prior = torch.distributions.Independent(
        torch.distributions.Normal(torch.zeros(10), torch.full((10,), float(np.sqrt(0.1)))), 1)
    core = ref.NPE_PFN_Core(prior=prior, regressor_init_kwargs={"random_state": RANDOM_STATE})
    core.append_simulations(theta, x)
    t0 = time.time()
    s, lp = core.sample_batched(x_obs, (N_SAMPLES,), with_log_prob=True)
    print(f"reference c5{' (full)' if full else '-structure'} sample_batched: {time.time() - t0:.1f} s, "
          f"{tuple(s.shape)}", flush=True)
    np.savez(os.path.join(HERE, "c5_full.npz" if full else "c5.npz"), theta=theta.numpy(), x=x.numpy(), x_obs=x_obs.numpy(), samples=s.numpy(),
             log_probs=lp.numpy(), random_state=RANDOM_STATE)


if __name__ == "__main__":
    main(full="--full" in sys.argv[1:])
