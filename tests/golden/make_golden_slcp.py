"""Golden vectors for config c3's call (SLCP, box prior, accept/reject) from the REFERENCE.

Run here (never on the GPU box -- /root/reference does not exist there):

    python tests/golden/make_golden_slcp.py

Loads the reference's npe_pfn.py / support_posterior.py / accept_reject_sampler.py by path with
the CPU oracle as ``tabpfn`` (as make_golden.py) and runs c3's call --
``TabPFN_Based_NPE_PFN(prior=BoxUniform(-3, 3)^5).sample((N,), x_o)`` on the sbibm SLCP task
(5 theta / 8 x, the prior's box rejection, 5 autoregressive dims, 8 estimators, the default
preprocessing ensemble) -- at a size the CPU oracle finishes in about a minute: 300 simulations
and 1000 posterior samples instead of 1000 and 10 000.  The task data come from
npe_pfn.tasks.slcp_task (a seeded input generator, stored in the fixture).  Writes
tests/golden/slcp.npz (data only): the simulations, x_o and the reference's samples and
log-probs, for tests/test_gpu_posterior.py's c3 C2ST / paired-draw checks.

``python tests/golden/make_golden_slcp.py --full [random_state ...]`` runs c3's call at its
configured context instead: all 1 000 SLCP simulations (tasks.slcp_task(1000, seed=0), the bench's
workload), 1 000 draws per random_state (default 31 and 47; the draw count is the only reduction,
the oracle's cost), the accept/reject batches of accept_reject_sampler.py:68-72 under the box
prior.  One fixture per random_state, tests/golden/c3_rs<k>.npz, for
tests/test_gpu_c3_posterior.py (C2ST / KS of independent draws, paired draws, log-prob).
"""

from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import REPO, _load_weights_module, install_reference  # noqa: E402

sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "npe-pfn_amd"))
from oracle.tabpfn_oracle import OracleRegressor  # noqa: E402

N_SIMS, N_SAMPLES, RANDOM_STATE = 300, 1000, 13
FULL_SIMS, FULL_STATES = 1000, (31, 47)


def main(full: bool = False, random_state: int = RANDOM_STATE):
    W = _load_weights_module()
    OracleRegressor.default_weights = W.synthetic_weights(W.ModelConfig(), seed=0)
    mods, BoxUniform = install_reference()
    ref = mods["npe_pfn"]
    # the task generator lives in the build's package; importing it after install_reference keeps
    # the reference's modules under "npe_pfn"
    import importlib.util
    spec = importlib.util.spec_from_file_location("npfn_tasks", os.path.join(REPO, "npe-pfn_amd", "npe_pfn", "tasks.py"))
    tasks = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tasks)
    theta, x, x_o = tasks.slcp_task(FULL_SIMS, seed=0) if full else tasks.slcp_task(N_SIMS, seed=4)
    prior = BoxUniform(torch.full((5,), -3.0), torch.full((5,), 3.0))
    post = ref.TabPFN_Based_NPE_PFN(prior=prior, regressor_init_kwargs={"random_state": random_state})
    post.append_simulations(theta, x)
    t0 = time.time()
    s, lp = post.sample((N_SAMPLES,), x=x_o, with_log_prob=True)
    print(f"reference c3{' (full)' if full else '-structure'} sample (random_state={random_state}): "
          f"{time.time() - t0:.1f} s, {tuple(s.shape)}", flush=True)
    name = f"c3_rs{random_state}.npz" if full else "slcp.npz"
    np.savez(os.path.join(HERE, name), theta=theta.numpy(), x=x.numpy(), x_o=x_o.numpy(), samples=s.numpy(),
             log_probs=lp.numpy(), random_state=random_state, low=np.full(5, -3.0, np.float32),
             high=np.full(5, 3.0, np.float32))


if __name__ == "__main__":
    if "--full" in sys.argv[1:]:
        for rs in ([int(a) for a in sys.argv[1:] if a != "--full"] or FULL_STATES):
            main(full=True, random_state=rs)
    else:
        main()
