"""Config c3's posterior against the reference's at c3's configured context: SLCP (5 theta / 8 x),
all 1 000 simulations (tasks.slcp_task(1000, seed=0), the bench's workload), the box prior
U(-3, 3)^5 with the accept/reject loop, the default std-Euclid filter, the default preprocessing
ensemble, 5 autoregressive dims, through ``TabPFN_Based_NPE_PFN.sample`` on the GPU, against the
reference's own ``TabPFN_Based_NPE_PFN.sample`` driving the CPU oracle (tests/golden/c3_rs<k>.npz,
made by ``tests/golden/make_golden_slcp.py --full`` from /root/reference/npe_pfn/npe_pfn.py:253-308,
708-744, accept_reject_sampler.py:9-91 and support_posterior.py:357-369; 1 000 draws per
random_state -- the oracle's cost, ~14 min each).  The rejection batches follow the reference's
recurrence (accept_reject_sampler.py:68-72) on both sides, so under the same random_state the
accepted draws pair up row by row as long as the same rows are rejected.

Tolerances (BASELINE.json north_star: "C2ST <= 0.55 vs reference"):

* independent draws (the GPU under one random_state, the reference under another): C2ST <= 0.55
  (tests/c2st.py, the reference's harness, scripts/evaluate_ropefm.py:119-280) and two-sample KS
  <= 0.087 per dimension (the alpha = 0.001 critical value at n = m = 1000);
* paired draws (same random_state, hence the same Philox uniforms at every AR step): median
  |theta_gpu - theta_ref| <= 2 % of the posterior std per dimension;
* log densities at fixed theta: the GPU's ``log_prob`` of the reference's draws within 0.05
  (median) of the reference's own ``with_log_prob`` values (pointwise, so a draw that a bf16
  difference moves across a low-density gap cannot hide or fake a difference).
"""
import os

import numpy as np
import pytest
import torch
from scipy.stats import ks_2samp

from c2st import c2st
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
STATES = (31, 47)


def _g(rs):
    return np.load(os.path.join(GOLDEN, f"c3_rs{rs}.npz"))


def _post(g, random_state):
    from npe_pfn.npe_pfn import TabPFN_Based_NPE_PFN
    from npe_pfn.tasks import slcp_prior

    post = TabPFN_Based_NPE_PFN(prior=slcp_prior(device=DEV),
                                regressor_init_kwargs={"random_state": random_state, "device": DEV})
    post.append_simulations(torch.from_numpy(g["theta"]).to(DEV), torch.from_numpy(g["x"]).to(DEV))
    return post


@pytest.fixture(scope="module")
def gpu_draws():
    out = {}
    for rs in STATES:
        g = _g(rs)
        s, lp = _post(g, rs).sample((1000,), x=torch.from_numpy(g["x_o"]).to(DEV), with_log_prob=True)
        out[rs] = (s.cpu().numpy(), lp.cpu().numpy())
    return out


def test_c3_golden_fixtures_share_the_task():
    a, b = _g(31), _g(47)
    assert np.array_equal(a["theta"], b["theta"]) and np.array_equal(a["x"], b["x"])
    assert a["theta"].shape == (1000, 5) and a["x"].shape == (1000, 8) and a["samples"].shape == (1000, 5)
    assert (np.abs(a["samples"]) <= 3.0).all() and (np.abs(b["samples"]) <= 3.0).all()
    assert np.isfinite(a["samples"]).all() and np.isfinite(a["log_probs"]).all()


@pytest.mark.parametrize("rs_gpu,rs_ref", [(47, 31), (31, 47)])
def test_c3_independent_draws_c2st_and_ks(gpu_draws, rs_gpu, rs_ref):
    s = gpu_draws[rs_gpu][0]
    ref = _g(rs_ref)["samples"]
    assert np.isfinite(s).all() and (np.abs(s) <= 3.0).all()
    ks = [ks_2samp(s[:, d], ref[:, d]).statistic for d in range(5)]
    assert max(ks) <= 0.087, ks
    score = c2st(s, ref, seed=1)
    print(f"c3 C2ST(gpu rs={rs_gpu}, reference rs={rs_ref}) = {score:.3f}; max KS {max(ks):.3f}")
    assert score <= 0.55, score


@pytest.mark.parametrize("rs", STATES)
def test_c3_paired_draws_match_reference(gpu_draws, rs):
    s = gpu_draws[rs][0]
    ref = _g(rs)["samples"]
    sd = ref.std(0)
    med = np.median(np.abs(s - ref), 0)
    print(f"c3 paired rs={rs}: median |d theta| / std per dim {np.round(med / sd, 4).tolist()}")
    assert (med <= 0.02 * sd).all(), (med / sd)


@pytest.mark.parametrize("rs", STATES)
def test_c3_log_prob_of_reference_draws(rs):
    g = _g(rs)
    lp = _post(g, rs).log_prob(torch.from_numpy(g["samples"]).to(DEV),
                               torch.from_numpy(g["x_o"]).to(DEV)).cpu().numpy()
    d = np.abs(lp - g["log_probs"])
    print(f"c3 log_prob rs={rs}: median |d| {np.median(d):.4f}, 95th pct {np.percentile(d, 95):.4f}")
    assert np.median(d) <= 0.05, np.median(d)
