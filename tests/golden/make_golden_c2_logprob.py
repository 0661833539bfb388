"""Golden vectors for the c2-size AR log-prob parity test (tests/test_gpu_c2_logprob.py).

The c2 workload's context -- Gaussian-linear 10D, 1 000 simulations (npe_pfn.tasks,
seed 0) -- through the fused AR log-prob path: for each of the 10 autoregressive steps
the CPU oracle (oracle/tabpfn_oracle.py, bf16-emulating, tabpfn's default preprocessing
ensemble, seed 2) fits on [x, theta_<k] -> theta_k and gives the bar log density of 48
query thetas at x_o (reference npe_pfn.py:462-524 teacher-forced sum; -inf -> log 1e-15
per dim).  Stored per step, with the context and queries, so the GPU test needs no oracle
run (the oracle takes minutes at this size).

This is test infrastructure: it runs the in-repo oracle, not the reference.
usage: python tests/golden/make_golden_c2_logprob.py  (writes tests/golden/c2_logprob.npz)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "npe-pfn_amd")]

from npe_pfn.tasks import gaussian_linear_task  # noqa: E402
from npe_pfn.weights import ModelConfig, synthetic_weights  # noqa: E402
from oracle.preprocess_oracle import MODE_ENSEMBLE  # noqa: E402
from oracle.tabpfn_oracle import OracleTabPFN, bar_nll  # noqa: E402


def main():
    cfg = ModelConfig()
    weights = synthetic_weights(cfg, seed=0)
    theta, x, x_o = (t.numpy() for t in gaussian_linear_task(10, 1000, seed=0))
    rng = np.random.default_rng(123)
    tq = np.concatenate([
        theta[rng.choice(1000, 40, replace=False)],                          # the prior's bulk
        theta[:1] * 0 + x_o * 0.5 + 0.05 * rng.normal(size=(7, 10)),         # near the posterior mean
        np.full((1, 10), 3.0),                                               # far tail: end bars
    ]).astype(np.float32)
    N = tq.shape[0]
    xq = np.repeat(x_o, N, 0).astype(np.float32)
    orc = OracleTabPFN(weights, cfg.n_estimators, cfg.softmax_temperature, seed=2, emulate_bf16=True,
                       preprocessing=MODE_ENSEMBLE)
    joint = np.concatenate([x, theta], 1)
    test = np.concatenate([xq, tq], 1)
    steps = np.zeros((10, N))
    for k in range(10):
        t0 = time.time()
        orc.fit(joint[:, : 10 + k], joint[:, 10 + k])
        p = orc.predict_probs(test[:, : 10 + k])
        d = -bar_nll(np.log(np.maximum(p, 1e-38)), orc.borders(), tq[:, k])
        steps[k] = np.where(np.isneginf(d), np.log(1e-15), d)
        print(f"step {k}: {time.time() - t0:.1f} s, mean log density {steps[k].mean():.3f}", flush=True)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "c2_logprob.npz"),
                        x=x, theta=theta, xq=xq, tq=tq, steps=steps)


if __name__ == "__main__":
    main()
