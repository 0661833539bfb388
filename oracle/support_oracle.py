"""CPU restatement of the support-side kernels -- TEST INFRASTRUCTURE ONLY.

Imported by tests/ as the checker of the HIP kernels in
npe-pfn_amd/csrc/npfn_support.hip; never by the product path.

* ``sir_select`` -- K11, the resampling step of PosteriorSupport.sample_sir
  (reference npe_pfn/support_posterior.py:216-241): truncate the prior log
  density where the posterior log density is below the threshold (:220), form
  the log importance ratios with ``torch.nan_to_num(., -inf)`` semantics (:223:
  NaN -> -inf, +inf -> FLT_MAX, -inf -> -FLT_MAX), normalise each group of
  ``k`` proposals with a log-sum-exp and report ESS = 1 / sum(p^2) (:228-232),
  and pick one proposal per group (:234-241).  The reference draws the pick
  with ``torch.distributions.Categorical`` (torch's global RNG); the engine and
  this restatement use the inverse CDF at u = Philox4x32-10(counter=(group,
  counter), key=seed), so the pick is exact against this restatement and
  equal in distribution to the reference.
* ``box_mask`` -- K10's mask (support_posterior.py:286-289).

Pinning: the orchestration around both (threshold, reshape, gather, loop) is
pinned by tests/golden/support.npz, produced by the reference's own
PosteriorSupport (tests/golden/make_golden_support.py); the Categorical draw
itself is torch-RNG specific, so the device pick is pinned only against this
restatement (parity of the draw: distributional).
"""

from __future__ import annotations

import numpy as np

from .philox import uniforms

FLT_MAX = np.float32(np.finfo(np.float32).max)


def log_ratios(lpr: np.ndarray, lq: np.ndarray, thr: float) -> np.ndarray:
    """support_posterior.py:220-223, float32 throughout."""
    lq = np.asarray(lq, dtype=np.float32)
    lpr = np.where(lq < np.float32(thr), np.float32(-np.inf), np.asarray(lpr, dtype=np.float32))
    with np.errstate(invalid="ignore", over="ignore"):
        d = (lpr - lq).astype(np.float32)
    nan = np.isnan(d)
    d = np.clip(d, -FLT_MAX, FLT_MAX)
    d[nan] = -np.inf
    return d.astype(np.float32)


def sir_select(lpr: np.ndarray, lq: np.ndarray, thr: float, k: int, seed: int, counter: int,
               group_offset: int = 0):
    """(pick [G] int64, ess [G] float32) for G = len(lq) // k groups."""
    lw = log_ratios(lpr, lq, thr).reshape(-1, k)
    G = lw.shape[0]
    u = uniforms(seed, counter, G, row_offset=group_offset).astype(np.float64)
    pick = np.zeros(G, dtype=np.int64)
    ess = np.zeros(G, dtype=np.float32)
    for g in range(G):
        row = lw[g]
        m = np.float32(row.max())
        if m == -np.inf:  # every ratio NaN: torch's probabilities are NaN
            ess[g] = np.nan
            continue
        with np.errstate(under="ignore", over="ignore", invalid="ignore"):
            e = np.exp((row - m).astype(np.float32)).astype(np.float64)
            s = e.sum()
            lse = np.float32(m + np.float32(np.log(np.float32(s))))
            p = np.exp((row - lse).astype(np.float32)).astype(np.float64)
        ess[g] = np.float32(1.0 / (p * p).sum())
        c = np.cumsum(e)
        j = int(np.searchsorted(c, u[g] * s, side="right"))
        if j >= k:  # u * s rounded past the total: last proposal with mass
            j = int(np.nonzero(e > 0)[0][-1])
        pick[g] = j
    return pick, ess


def box_mask(theta: np.ndarray, lower: np.ndarray, upper: np.ndarray) -> np.ndarray:
    """support_posterior.py:286-288: all((s >= lower) & (s <= upper), dim=1)."""
    return np.all((theta >= lower) & (theta <= upper), axis=1)
