"""Golden predictive distribution of a 500-feature table under the default ensemble (the oracle).

    python tests/golden/make_golden_wide.py      (~28 min on 8 cores; the oracle only, no reference)

tabpfn takes up to 500 features without ``ignore_pretraining_limits`` [ext: tabpfn 2.2.1]; under
the regressor's default preprocessing ensemble the quantile + original + SVD pipeline then has
2 * 500 + 11 + 1 = 1012 features (507 tokens per row) at 100 context rows, the power + fingerprint
pipeline 501 (252 tokens).  The CPU oracle (oracle/tabpfn_oracle.py, bf16-emulating, the full
12-layer synthetic model of ModelConfig(), weights seed 0, random_state 3) predicts 16 query rows;
its cost (~2 min per layer here) keeps it out of a GPU test, so the test reads this fixture.
Writes tests/golden/wide500.npz: X [116, 500] (100 context rows, then the queries), y [100],
probs [16, 5000] (float32).
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "npe-pfn_amd"))

from npe_pfn.weights import ModelConfig, synthetic_weights  # noqa: E402
from oracle.tabpfn_oracle import OracleTabPFN  # noqa: E402

F, N_CTX, N_Q, SEED = 500, 100, 16, 3


def table():
    rng = np.random.default_rng(F)
    z = rng.normal(size=(N_CTX + N_Q, 3))
    X = (z @ rng.normal(size=(3, F)) + 0.3 * rng.normal(size=(N_CTX + N_Q, F))).astype(np.float32)
    y = (z[:N_CTX, 0] + 0.2 * rng.normal(size=N_CTX)).astype(np.float32)
    return X, y


def main():
    cfg = ModelConfig()
    w = synthetic_weights(cfg, seed=0)
    X, y = table()
    orc = OracleTabPFN(w, cfg.n_estimators, cfg.softmax_temperature, seed=SEED, emulate_bf16=True, preprocessing=3)
    orc.fit(X[:N_CTX], y)
    p = orc.predict_probs(X[N_CTX:]).astype(np.float32)
    assert np.isfinite(p).all()
    np.savez_compressed(os.path.join(HERE, "wide500.npz"), X=X, y=y, probs=p, random_state=SEED)
    print("wrote wide500.npz", p.shape)


if __name__ == "__main__":
    main()
