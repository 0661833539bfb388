"""The C2ST harness itself (CPU): 0.5 on two draws of one law, near 1 on separated laws."""
import numpy as np

from c2st import c2st


def test_same_distribution_scores_near_half():
    rng = np.random.default_rng(0)
    a = rng.normal(size=(600, 2))
    b = rng.normal(size=(600, 2))
    assert abs(c2st(a, b, epochs=30) - 0.5) < 0.05


def test_shifted_distribution_is_detected():
    rng = np.random.default_rng(1)
    a = rng.normal(size=(600, 2))
    b = rng.normal(size=(600, 2)) + np.array([1.5, 0.0])
    assert c2st(a, b, epochs=30) > 0.7
