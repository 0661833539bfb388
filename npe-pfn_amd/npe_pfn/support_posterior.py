"""Truncated-proposal support, box pre-rejection and context filters.

Reference: npe_pfn/support_posterior.py (PosteriorSupport :13-258,
prereject_with_bounds :264-309, check_for_uniform :312-318, filters
:327-369).  Filters keep the reference semantics (pinned by
tests/golden/filters.npz); when the simulation table lives on the GPU the
standardized-Euclidean filter runs as the K12 kernel ``npfn_filter_stdeuclid``.
"""

from __future__ import annotations

import logging
from typing import Any, Mapping, Optional

import torch
from torch import Tensor
from torch.distributions import Independent, Uniform
from tqdm.auto import tqdm

log = logging.getLogger(__name__)


def BoxUniform(low, high) -> Independent:
    """Box prior equivalent to ``sbi.utils.BoxUniform`` (sbi 0.23.3)."""
    low = torch.as_tensor(low, dtype=torch.float32)
    high = torch.as_tensor(high, dtype=torch.float32)
    return Independent(Uniform(low, high), 1)


class PosteriorSupport:
    """HPD-truncated prior used as the next-round proposal of TSNPE-PFN."""

    def __init__(
        self,
        prior: Any,
        posterior: Any,
        obs: Tensor,
        num_samples_to_estimate_support: int = 10_000,
        batch_size_for_estimate_support: int = 10_000,
        allowed_false_negatives: float = 0.0,
        sampling_method: str = "rejection",
        max_iter_rejection: int = 1000,
        oversample_sir: int = 100,
        log_prob_kwargs: Mapping = {},
    ) -> None:
        self._prior = prior
        self._posterior = posterior
        self._obs = obs
        self._posterior_thr = None
        self.sampling_method = sampling_method
        self.max_iter = max_iter_rejection
        self.oversample_sir = oversample_sir
        self.allowed_false_negatives = allowed_false_negatives
        self._log_prob_kwargs = dict(log_prob_kwargs)
        if sampling_method == "rejection":
            draws = self._posterior.sample((num_samples_to_estimate_support,), self._obs,
                                           max_sampling_batch_size=batch_size_for_estimate_support)
            self.thr = self.tune_threshold(draws, allowed_false_negatives, batch_size=batch_size_for_estimate_support)

    def tune_threshold(self, samples: Tensor, allowed_false_negatives: float = 0.0, batch_size: int = 10_000):
        lp = self._posterior.log_prob(samples, self._obs, max_sampling_batch_size=batch_size, **self._log_prob_kwargs)
        return torch.quantile(lp, allowed_false_negatives)

    def sample(self, sample_shape: torch.Size = torch.Size(), show_progress_bars: bool = True,
               sampling_batch_size: int = 10_000, return_acceptance_rate: bool = False, return_ess: bool = False):
        if self.sampling_method == "rejection":
            return self.sample_rejection(sample_shape, show_progress_bars, sampling_batch_size, return_acceptance_rate)
        if self.sampling_method == "sir":
            return self.sample_sir(sample_shape, show_progress_bars, sampling_batch_size, return_ess)
        raise ValueError(f"Unknown sampling method: {self.sampling_method}")

    def sample_rejection(self, sample_shape=torch.Size(), show_progress_bars: bool = True,
                         sampling_batch_size: int = 10_000, return_acceptance_rate: bool = False):
        """Prior draws kept where log q(theta|x_o) > threshold (reference :97-182)."""
        shape = torch.Size(sample_shape)
        assert len(shape) == 1
        n = shape[0]
        bar = tqdm(disable=not show_progress_bars, total=n, desc=f"Drawing {n} restricted posterior samples")
        pre_rate = 1.0
        low = high = None
        proposed, remaining = 0, n
        kept = []
        for _ in range(self.max_iter):
            if remaining <= 0:
                break
            if low is None or high is None:
                cand = self._prior.sample((sampling_batch_size,))
                lp = self._posterior.log_prob(cand, self._obs, **self._log_prob_kwargs)
                low, high = self._posterior._get_classifier_bounds()
            else:
                cand, pre_rate = prereject_with_bounds(self._prior, low, high, sampling_batch_size)
                lp = self._posterior.log_prob(cand, self._obs, **self._log_prob_kwargs)
                lo2, hi2 = self._posterior._get_classifier_bounds()
                assert torch.allclose(low, lo2) and torch.allclose(high, hi2)
            acc = cand[(lp > self.thr).bool()]
            kept.append(acc)
            proposed += sampling_batch_size
            remaining -= acc.shape[0]
            bar.update(acc.shape[0])
        bar.close()
        rate = (n - remaining) / proposed
        log.info(f"Pre-acceptance rate: {pre_rate}")
        log.info(f"Log prob acceptance rate: {rate}")
        overall = pre_rate * rate
        log.info(f"Overall acceptance rate: {overall}")
        if remaining > 0:
            extra = self._prior.sample((remaining,))
            kept.append(extra)
            log.info(f"Max iter exceeded. Added {extra} prior samples.")
        out = torch.cat(kept)[:n]
        assert out.shape[0] == n
        return (out, overall) if return_acceptance_rate else out

    def sample_sir(self, sample_shape=torch.Size(), show_progress_bars: bool = True,
                   sampling_batch_size: int = 10_000, return_ess: bool = False):
        """Sampling-importance-resampling from the posterior (reference :184-258)."""
        shape = torch.Size(sample_shape)
        assert len(shape) == 1
        n = shape[0]
        bar = tqdm(disable=not show_progress_bars, total=n, desc=f"Drawing {n} restricted posterior samples")
        k = self.oversample_sir
        assert sampling_batch_size % k == 0
        groups = sampling_batch_size // k
        remaining = n
        out, ess_all = [], []
        while remaining > 0:
            th, lq = self._posterior.sample((sampling_batch_size,), self._obs,
                                            max_sampling_batch_size=sampling_batch_size, with_log_prob=True)
            lpr = self._prior.log_prob(th)
            thr = torch.quantile(lq, self.allowed_false_negatives)
            if th.is_cuda:
                # K11 on the device: truncation, log ratios, ESS, pick and gather in one launch;
                # the pick's uniforms are Philox keyed by a seed from torch's global RNG
                seed = int(torch.randint(0, 2**62, (1,)).item())
                sel, _, ess = sir_select(th, lpr, lq, thr, k, seed)
                ess_all.append(ess)
                out.append(sel)
                remaining -= groups
                bar.update(groups)
                continue
            lpr[lq < thr] = -float("inf")
            lw = torch.nan_to_num(lpr - lq, -float("inf")).reshape(groups, k)
            w = torch.exp(lw - torch.logsumexp(lw, dim=1, keepdim=True))
            ess_all.append(1.0 / torch.sum(w**2, dim=1))
            pick = torch.distributions.Categorical(logits=lw).sample((1,))[0, :]
            out.append(th.reshape(groups, k, -1)[torch.arange(groups), pick])
            remaining -= groups
            bar.update(groups)
        bar.close()
        samples = torch.cat(out)[:n]
        assert samples.shape[0] == n
        ess = torch.cat(ess_all)
        log.info(f"Mean ESS: {ess.mean().item()}")
        log.info(f"Min ESS: {ess.min().item()}")
        return (samples, ess) if return_ess else samples


def prereject_with_bounds(proposal: Any, lower_bound: Tensor, upper_bound: Tensor, sampling_batch_size: int = 10_000,
                          pre_sampling_batch_size: int = 1_000_000):
    """Draws from ``proposal`` restricted to the box [lower, upper] (reference :264-309)."""
    uniform = check_for_uniform(proposal)
    n_acc = 0
    n_tot = 0
    pieces = []
    while n_acc < sampling_batch_size:
        s = proposal.sample((pre_sampling_batch_size,))
        if s.is_cuda:
            s = box_compact(s, lower_bound, upper_bound)  # K9 mask + K10 ordered compaction
        else:
            inside = torch.all((s >= lower_bound) & (s <= upper_bound), dim=1)
            s = s[inside.bool()]
        pieces.append(s)
        n_acc += s.shape[0]
        n_tot += pre_sampling_batch_size
        if uniform:
            break
    rate = n_acc / n_tot
    if uniform:
        plo, phi = get_uniform_bounds(proposal)
        return BoxUniform(torch.max(lower_bound, plo), torch.min(upper_bound, phi)).sample((sampling_batch_size,)), rate
    return torch.cat(pieces)[:sampling_batch_size], rate


def _lib_stream(device):
    import ctypes

    from .engine import load_library

    return load_library(), ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def sir_select(theta: Tensor, lpr: Tensor, lq: Tensor, thr: Tensor, k: int, seed: int, counter: int = 0):
    """K11 ``npfn_sir_select``: (theta of the picks [G, D], pick [G], ess [G]), G = len(lq) // k.

    Device tensors only (the library raises without a GPU)."""
    from .engine import _check, _ptr

    dev = lq.device
    lib, stream = _lib_stream(dev)

    def f32(t):
        return torch.as_tensor(t).to(device=dev, dtype=torch.float32).contiguous()

    th, a, b, t = f32(theta), f32(lpr).reshape(-1), f32(lq).reshape(-1), f32(thr).reshape(1)
    if b.shape[0] % k or a.shape != b.shape or th.shape[0] != b.shape[0]:
        raise ValueError("sir_select: proposals must form whole groups of k with matching log densities")
    G, D = b.shape[0] // k, th.shape[1]
    pick = torch.empty(G, dtype=torch.int64, device=dev)
    ess = torch.empty(G, dtype=torch.float32, device=dev)
    out = torch.empty(G, D, dtype=torch.float32, device=dev)
    _check(lib, lib.npfn_sir_select(_ptr(a), _ptr(b), _ptr(t), G, int(k), int(seed) & (2**64 - 1), int(counter), 0,
                                    _ptr(th), D, _ptr(pick), _ptr(ess), _ptr(out), stream), "npfn_sir_select")
    return out, pick, ess


def box_compact(s: Tensor, lower: Tensor, upper: Tensor) -> Tensor:
    """Rows of ``s`` inside [lower, upper] in order: K9 ``npfn_box_support`` + K10 ``npfn_compact_rows``."""
    from .engine import _check, _ptr

    dev = s.device
    lib, stream = _lib_stream(dev)
    src = s.to(torch.float32).contiguous()
    n, D = src.shape
    if n == 0:
        return src
    lo = torch.as_tensor(lower).to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
    hi = torch.as_tensor(upper).to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
    mask = torch.empty(n, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    _check(lib, lib.npfn_box_support(_ptr(src), n, D, _ptr(lo), _ptr(hi), _ptr(mask), stream), "npfn_box_support")
    _check(lib, lib.npfn_compact_rows(_ptr(src), _ptr(mask), n, D, _ptr(dst), _ptr(cnt), stream), "npfn_compact_rows")
    return dst[: int(cnt.item())]


def check_for_uniform(proposal: Any) -> bool:
    return isinstance(proposal, Independent) and isinstance(proposal.base_dist, Uniform)


def get_uniform_bounds(proposal):
    return proposal.base_dist.low, proposal.base_dist.high


# ----------------------------------------------------------------- filters
# Every filter returns (theta, x) in that order (reference :326).
def get_filtering_method(name):
    table = {
        "no_filtering": no_filtering,
        "latest_filtering": latest_filtering,
        "random_filtering": random_filtering,
        "standardized_euclidean_filtering": standardized_euclidean_filtering,
    }
    if isinstance(name, str) and name in table:
        return table[name]
    if callable(name):
        return name
    raise ValueError(f"Unknown filtering method: {name}")


def no_filtering(obs: Tensor, theta: Tensor, x: Tensor, context_size: int):
    return theta, x


def latest_filtering(obs: Tensor, theta: Tensor, x: Tensor, context_size: int):
    return theta[-context_size:], x[-context_size:]


def random_filtering(obs: Tensor, theta: Tensor, x: Tensor, context_size: int):
    order = torch.randperm(theta.shape[0])
    keep = order[:context_size]
    return theta[keep], x[keep]


def standardized_euclidean_filtering(obs: Tensor, theta: Tensor, x: Tensor, context_size: int):
    """The ``context_size`` simulations closest to ``obs`` in z-scored Euclidean distance."""
    k = min(context_size, x.shape[0])
    if x.is_cuda:
        from .engine import Engine  # noqa: F401  (library must be present on GPU runs)
        from .engine import load_library, _check, _ptr

        lib = load_library()
        xs = x.to(torch.float32).contiguous()
        ob = obs.reshape(-1).to(device=x.device, dtype=torch.float32).contiguous()
        idx = torch.empty(k, dtype=torch.int64, device=x.device)
        import ctypes

        stream = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
        _check(lib, lib.npfn_filter_stdeuclid(_ptr(xs), xs.shape[0], xs.shape[1], _ptr(ob), k, _ptr(idx), stream),
               "npfn_filter_stdeuclid")
        return theta[idx], x[idx]
    mean = x.mean(dim=0)
    std = x.std(dim=0)
    dist = torch.norm((x - mean) / std - (obs - mean) / std, dim=1)
    _, idx = torch.topk(dist, k, largest=False)
    return theta[idx], x[idx]
