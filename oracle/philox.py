"""ORACLE (test infrastructure only) -- counter-based RNG shared with the engine.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this package.  The product path never does.

Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3",
SC'11) and splitmix64 (Steele et al. 2014), restated in numpy.  The reference
draws the bar-distribution uniforms from torch's global CPU RNG inside
``criterion.sample`` [ext: tabpfn 2.2.1 BarDistribution.sample, called at
npe_pfn/npe_pfn.py:146,220]; the engine replaces that stream with
``u(seed, counter, row)`` below so GPU and oracle draw identical uniforms.
Pinned by the Random123 known-answer vectors in tests/test_oracle_rng.py.
"""

from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32 with 10 rounds. All inputs uint32 arrays/scalars."""
    c0 = np.asarray(c0, dtype=np.uint32).astype(np.uint64)
    c1 = np.asarray(c1, dtype=np.uint32).astype(np.uint64)
    c2 = np.asarray(c2, dtype=np.uint32).astype(np.uint64)
    c3 = np.asarray(c3, dtype=np.uint32).astype(np.uint64)
    k0 = np.asarray(k0, dtype=np.uint32).astype(np.uint64)
    k1 = np.asarray(k1, dtype=np.uint32).astype(np.uint64)
    for r in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & _MASK32, lo1, (hi0 ^ c3 ^ k1) & _MASK32, lo0
        if r < 9:
            k0 = (k0 + np.uint64(W0)) & _MASK32
            k1 = (k1 + np.uint64(W1)) & _MASK32
    return (c0.astype(np.uint32), c1.astype(np.uint32), c2.astype(np.uint32), c3.astype(np.uint32))


def uniforms(seed: int, counter: int, n: int, row_offset: int = 0) -> np.ndarray:
    """u(seed, counter, row) in [0, 1): float32, 24 random bits.

    counter block = (row_lo, row_hi, counter_lo, counter_hi), key = (seed_lo, seed_hi).
    """
    rows = np.arange(row_offset, row_offset + n, dtype=np.uint64)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    counter = int(counter) & 0xFFFFFFFFFFFFFFFF
    x0, _, _, _ = philox4x32_10(
        (rows & _MASK32).astype(np.uint32),
        (rows >> np.uint64(32)).astype(np.uint32),
        np.uint32(counter & 0xFFFFFFFF),
        np.uint32(counter >> 32),
        np.uint32(seed & 0xFFFFFFFF),
        np.uint32(seed >> 32),
    )
    return ((x0 >> np.uint32(8)).astype(np.float32) * np.float32(2.0**-24)).astype(np.float32)


_GOLD = 0x9E3779B97F4A7C15
_U64 = (1 << 64) - 1


def splitmix64_next(state: int):
    """Returns (new_state, output)."""
    state = (state + _GOLD) & _U64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _U64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _U64
    return state, z ^ (z >> 31)


def estimator_permutation(seed: int, estimator: int, n_features: int) -> np.ndarray:
    """Per-estimator feature permutation (Fisher-Yates on splitmix64).

    Stands in for tabpfn's per-estimator feature shuffle [ext: tabpfn 2.2.1
    ensemble config, FEATURE_SHIFT_METHOD "shuffle"].
    """
    s = (int(seed) & 0xFFFFFFFF) | ((estimator & 0xFFFF) << 32) | ((n_features & 0xFFFF) << 48)
    p = list(range(n_features))
    for i in range(n_features - 1, 0, -1):
        s, out = splitmix64_next(s)
        j = out % (i + 1)
        p[i], p[j] = p[j], p[i]
    return np.asarray(p, dtype=np.int64)


CLASS_SALT = 0x5A17C1A55E5EED00


def class_permutation(seed: int, estimator: int, n_classes: int) -> np.ndarray:
    """Per-estimator class-label permutation of the classifier ensemble.

    Stands in for tabpfn's per-estimator class shift [ext: tabpfn 2.2.1
    ensemble config, CLASS_SHIFT_METHOD "shuffle"]; same Fisher-Yates as
    ``estimator_permutation`` on a salted state (npfn_kernels.hip k_class_params).
    """
    s = ((int(seed) & 0xFFFFFFFF) | ((estimator & 0xFFFF) << 32) | ((n_classes & 0xFFFF) << 48)) ^ CLASS_SALT
    p = list(range(n_classes))
    for i in range(n_classes - 1, 0, -1):
        s, out = splitmix64_next(s)
        j = out % (i + 1)
        p[i], p[j] = p[j], p[i]
    return np.asarray(p, dtype=np.int64)
