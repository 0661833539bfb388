"""GPU parity of the classifier path through the C-ABI.

``npfn_fit_classes`` / ``npfn_predict_proba`` (TabPFNClassifier.fit/predict_proba,
npe_pfn.py:661, :697) against the CPU oracle (OracleTabPFN.fit_classes /
predict_proba), and the ratio-based log density (DensityRatioWrapper,
npe_pfn.py:603-704) on the engine classifier against the same wrapper driven by
the oracle classifier.

Tolerances (floating point; bf16 GEMM/attention operands, fp32 accumulation):
* class probabilities: max |dp| <= 0.01 against the bf16-emulating oracle,
  <= 0.03 against the fp32 oracle;
* ratio log density: |d log q| <= 0.05 where both classifiers see the same
  training set (identical posterior and uniform samples).
"""
import numpy as np
import pytest
import torch

from npe_pfn.weights import classifier_config, synthetic_classifier_weights
from oracle.tabpfn_oracle import OracleClassifier, OracleTabPFN

pytestmark = pytest.mark.gpu

CFG = classifier_config()


@pytest.fixture(scope="module")
def cweights():
    return synthetic_classifier_weights(CFG, seed=1)


@pytest.fixture(scope="module")
def cengine(cweights):
    from npe_pfn.engine import Engine

    return Engine(CFG, cweights, device=torch.device("cuda", 0), random_state=4, preprocessing="none")


def _cls_data(n, F, K, N, seed):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, F)).astype(np.float32)
    score = X @ rng.normal(size=F)
    y = np.digitize(score, np.quantile(score, np.linspace(0, 1, K + 1)[1:-1])).astype(np.int64)
    Xq = rng.normal(size=(N, F)).astype(np.float32)
    return X, y, Xq


@pytest.mark.parametrize("n,F,K,N", [(150, 2, 2, 60), (90, 3, 3, 45), (61, 5, 4, 33)])
def test_predict_proba_matches_oracle(cengine, cweights, n, F, K, N):
    X, y, Xq = _cls_data(n, F, K, N, seed=n + F + K)
    cengine.fit_classes(torch.from_numpy(X), torch.from_numpy(y).float(), K)
    p_gpu = cengine.predict_proba(torch.from_numpy(Xq)).cpu().numpy()
    assert p_gpu.shape == (N, K)
    np.testing.assert_allclose(p_gpu.sum(1), 1.0, atol=1e-5)
    for emulate, tol in ((True, 0.01), (False, 0.03)):
        orc = OracleTabPFN(cweights, CFG.n_estimators, CFG.softmax_temperature, seed=4, emulate_bf16=emulate)
        orc.fit_classes(X, y, K)
        p_ref = orc.predict_proba(Xq)
        err = np.abs(p_gpu - p_ref).max()
        assert err <= tol, (emulate, err)


def test_classifier_surface_label_encoding(cweights):
    """TabPFNClassifier: arbitrary labels -> sorted classes_, numpy probabilities (npe_pfn.py:697)."""
    from npe_pfn.tabpfn import TabPFNClassifier

    X, y, Xq = _cls_data(80, 2, 2, 20, seed=7)
    labels = np.where(y == 1, 5.0, -1.0).astype(np.float32)  # non-index labels
    clf = TabPFNClassifier(random_state=4, weights=cweights, device="cuda:0")
    clf.fit(torch.from_numpy(X), torch.from_numpy(labels))
    assert list(clf.classes_) == [-1.0, 5.0]
    p = clf.predict_proba(torch.from_numpy(Xq))
    assert isinstance(p, np.ndarray) and p.shape == (20, 2)
    orc = OracleClassifier(random_state=4, weights=cweights, emulate_bf16=True, preprocessing="ensemble")
    orc.fit(torch.from_numpy(X), torch.from_numpy(labels))
    assert np.abs(p - orc.predict_proba(torch.from_numpy(Xq))).max() <= 0.01


def test_ratio_log_probs_match_oracle_classifier(cweights):
    from npe_pfn.npe_pfn import DensityRatioWrapper

    rng = np.random.default_rng(3)
    post = torch.from_numpy((rng.normal(size=(300, 2)) * [0.2, 0.4] + [0.1, -0.3]).astype(np.float32))
    theta = torch.from_numpy((rng.normal(size=(120, 2)) * 0.6).astype(np.float32))
    x = torch.zeros(1, 2)
    out = []
    for backend in ("engine", "oracle"):
        w = DensityRatioWrapper(random_state=4, weights=cweights, device="cuda:0")
        if backend == "oracle":
            w._classifier = OracleClassifier(random_state=4, weights=cweights, emulate_bf16=True,
                                             preprocessing="ensemble")
        torch.manual_seed(99)  # same uniform samples for both classifiers
        w.fit(x, post, 0.1, post, post)
        out.append(w.ratio_log_probs(theta.cuda() if backend == "engine" else theta).cpu().numpy())
    inside = np.all((theta.numpy() >= w._padded_dim_min.numpy()) & (theta.numpy() <= w._padded_dim_max.numpy()), 1)
    assert inside.any() and (~inside).any()
    np.testing.assert_allclose(out[0][~inside], out[1][~inside], rtol=1e-6)
    assert np.abs(out[0] - out[1]).max() <= 0.05


def test_classifier_c4_context_size(cengine):
    """c4 shape: 10 000-row classifier context (5 000 uniform + 5 000 posterior), 2 features."""
    g = torch.Generator(device="cuda").manual_seed(0)
    post = torch.randn(5000, 2, device="cuda", generator=g) * 0.1 + 0.5
    unif = torch.rand(5000, 2, device="cuda", generator=g) * 2 - 1
    X = torch.cat([unif, post])
    y = torch.cat([torch.zeros(5000, device="cuda"), torch.ones(5000, device="cuda")])
    cengine.fit_classes(X, y, 2)
    q = torch.cat([post[:500], unif[:500]])
    p = cengine.predict_proba(q)
    assert torch.isfinite(p).all()
    torch.testing.assert_close(p.sum(1), torch.ones(1000, device="cuda"), atol=1e-5, rtol=0)


def test_classifier_ensemble_c4_context_size(cweights):
    """c4's classifier context (5 000 uniform + 5 000 posterior rows) under the default
    ensemble preprocessing (fingerprint limit: 10 000 rows): finite, normalised probabilities,
    and the posterior rows score above the uniform ones."""
    from npe_pfn.tabpfn import TabPFNClassifier

    g = torch.Generator(device="cuda").manual_seed(0)
    post = torch.randn(5000, 2, device="cuda", generator=g) * 0.1 + 0.5
    unif = torch.rand(5000, 2, device="cuda", generator=g) * 2 - 1
    X = torch.cat([unif, post])
    y = torch.cat([torch.zeros(5000, device="cuda"), torch.ones(5000, device="cuda")])
    clf = TabPFNClassifier(random_state=4, device="cuda:0", weights=cweights)
    assert clf.preprocessing == "ensemble"
    clf.fit(X, y)
    p = clf.predict_proba_tensor(torch.cat([post[:500], unif[:500]]))
    assert torch.isfinite(p).all()
    torch.testing.assert_close(p.sum(1), torch.ones(1000, device="cuda"), atol=1e-5, rtol=0)


def test_regressor_predict_refused_after_classifier_fit(cengine):
    from npe_pfn.engine import EngineError

    X, y, Xq = _cls_data(40, 2, 2, 5, seed=1)
    cengine.fit_classes(torch.from_numpy(X), torch.from_numpy(y).float(), 2)
    with pytest.raises(EngineError, match="classifier fit"):
        cengine.predict_logits(torch.from_numpy(Xq))


def test_tsnpe_two_moons_ratio_based_c4_small():
    """c4 in miniature: TSNPE-PFN rounds with the ratio-based log density (tsnpe_pfn.py:14-119)."""
    from npe_pfn import run_tsnpe_pfn
    from npe_pfn.tasks import two_moons_prior, two_moons_simulator

    torch.manual_seed(42)
    prior = two_moons_prior()
    x_o = two_moons_simulator(0.5 * torch.ones(1, 2))
    post = run_tsnpe_pfn(two_moons_simulator, prior, x_o, num_simulations=200, num_rounds=2,
                         proposal_batch_size=500, simulation_batch_size=100,
                         num_samples_to_estimate_support=1000)
    assert post._theta_train.shape[0] == 200
    s = post.sample((300,), x=x_o)
    assert s.shape == (300, 2) and torch.isfinite(s).all()
    assert ((s >= -1) & (s <= 1)).all()
    lp = post.log_prob(s[:50].cpu(), x_o, mode="ratio_based", num_posterior_samples=1000)
    assert torch.isfinite(lp).all()


@pytest.mark.parametrize("mode,pre,n", [("quantile", 1, 180), ("quantile+power", 2, 180), ("ensemble", 3, 180),
                                        ("ensemble", 3, 2000)])
def test_predict_proba_with_preprocessing_matches_oracle(cweights, mode, pre, n):
    """Classifier engine with feature preprocessing (npfn_set_preprocessing) vs the oracle
    with the same mode; tolerance as the plain classifier test (bf16-emulating: 0.01).
    "ensemble" is the classifier's default: tabpfn's coarse-quantile + original + SVD | original
    pipelines with the fingerprint feature [ext], restated in oracle/preprocess_oracle.py."""
    from npe_pfn.tabpfn import TabPFNClassifier

    X, y, Xq = _cls_data(n, 3, 2, 50, seed=17)
    X[:, 0] = np.exp(1.5 * X[:, 0])
    Xq[:, 0] = np.exp(1.5 * Xq[:, 0])
    clf = TabPFNClassifier(random_state=4, device="cuda:0", weights=cweights, preprocessing=mode)
    clf.fit(torch.from_numpy(X), torch.from_numpy(y))
    p_gpu = clf.predict_proba(torch.from_numpy(Xq))
    orc = OracleTabPFN(cweights, CFG.n_estimators, CFG.softmax_temperature, seed=4, emulate_bf16=True,
                       preprocessing=pre)
    orc.fit_classes(X, y, 2)
    err = np.abs(np.asarray(p_gpu) - orc.predict_proba(Xq)).max()
    assert err <= 0.01, err
