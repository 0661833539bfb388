"""NPE-PFN estimators (reference: npe_pfn/npe_pfn.py).

Public surface kept from the reference: ``NPE_PFN_Core`` (:26-600) and
``TabPFN_Based_NPE_PFN`` (:708-744) with ``append_simulations``, ``sample``,
``sample_batched``, ``log_prob`` and pickling.  The autoregressive loop
(``_sample`` :111-169, ``_sample_batched`` :171-251,
``_autoregressive_log_prob`` :462-524) has two implementations:

* **fused** -- when the estimator offers ``ar_sample`` / ``ar_log_prob``
  (the engine-backed :class:`npe_pfn.tabpfn.TabPFNRegressor`), the whole
  dimension loop runs on the GPU in one C-ABI call (``npfn_ar_sample``):
  context and samples stay in HBM, each step's fit is computed once;
* **generic** -- any object with the tabpfn ``fit`` / ``predict`` /
  ``criterion`` surface is driven step by step exactly like the reference.

Both produce the same numbers for the same estimator (tests/test_orchestration.py
pins the generic loop to golden vectors made by the reference itself).
"""

from __future__ import annotations

import contextlib
import math
from typing import Callable, Mapping, Optional, Tuple, Union

import torch
from torch import Tensor
from torch.distributions import Distribution

from .accept_reject_sampler import accept_reject_sample
from .support_posterior import (get_filtering_method, latest_filtering, no_filtering,
                                standardized_euclidean_filtering)
from .tabpfn import TabPFNClassifier, TabPFNRegressor


DETERMINISTIC_FILTERS = (no_filtering, latest_filtering, standardized_euclidean_filtering)


class NPE_PFN_Core:
    """Training-free neural posterior estimation with a tabular foundation model."""

    def __init__(
        self,
        show_progress_bars: bool = False,
        prior: Optional[Distribution] = None,
        embedding_net: Optional[torch.nn.Module] = None,
        x_shape: Optional[torch.Size] = None,
        regressor_init_kwargs: Mapping = {},
        classifier_init_kwargs: Mapping = {},
    ) -> None:
        self.show_progress_bars = show_progress_bars
        self.prior = prior
        self.embedding_net = embedding_net
        self.x_shape = x_shape
        self.regressor_init_kwargs = dict(regressor_init_kwargs)
        self.classifier_init_kwargs = dict(classifier_init_kwargs)
        self._model = TabPFNRegressor(**self.regressor_init_kwargs)
        self._model_classifier = None
        self._obs_offset = 0  # first observation index of this process's shard (npe_pfn.distributed)
        self._theta_train: Optional[Tensor] = None
        self._x_train: Optional[Tensor] = None

    # ------------------------------------------------------------- pickling
    def __getstate__(self):
        # the estimators hold device state; they are rebuilt on load (reference :57-71)
        state = dict(self.__dict__)
        state["_model"] = None
        state["_model_classifier"] = None
        return state

    def __setstate__(self, state):
        self.__dict__.update(state)
        self._model = TabPFNRegressor(**self.regressor_init_kwargs)

    # ------------------------------------------------------------- data
    def _embed(self, x: Tensor) -> Tensor:
        if self.embedding_net is None:
            return x
        return self.embedding_net(x.reshape(-1, *self.x_shape))

    def append_simulations(self, theta: Tensor, x: Tensor):
        """Replace the context table by (theta, x) (reference :73-82)."""
        self._theta_train = None
        self._x_train = None
        x = self._embed(x)
        self._theta_train = self._validate_theta(theta)
        self._x_train = self._validate_x(x)
        return self

    def get_context(self, x: Tensor) -> Tuple[Tensor, Tensor]:
        return self._theta_train, self._x_train

    def _validate_x(self, x: Tensor) -> Tensor:
        if x is None:
            raise NotImplementedError("Setting a default x is not yet supported.")
        if x.ndim == 1:
            x = x.unsqueeze(0)
        assert x.ndim == 2, "x must be a 2D tensor."
        if self._x_train is not None:
            assert x.shape[1] == self._x_train.shape[1], "The number of features in x must match the training data."
        return x

    def _validate_theta(self, theta: Tensor) -> Tensor:
        if theta.ndim == 1:
            theta = theta.unsqueeze(0)
        assert theta.ndim == 2, "theta must be a 2D tensor."
        if self._theta_train is not None:
            assert theta.shape[1] == self._theta_train.shape[1], \
                "The number of features in theta must match the training data."
        return theta

    def _fused(self) -> bool:
        return hasattr(self._model, "ar_sample")

    def _context_is_deterministic(self) -> bool:
        """Whether get_context(x) returns the same table every time it is called with the same x."""
        return True

    def _reuse_fits(self):
        """One context for the block (one sample / sample_batched / log_prob call): the engine
        keeps every AR step's fit across the accept/reject batches instead of refitting.
        Only when the context is a deterministic function of x: a random filter draws a new
        subset per batch and the reference refits on each (npe_pfn.py:128, support_posterior.py:351)."""
        ctx = getattr(self._model, "reuse_fits", None)
        if ctx is None or not self._context_is_deterministic():
            return contextlib.nullcontext()
        return ctx()

    # --------------------------------------------------- autoregressive core
    def _ar_generic(self, x_ctx: Tensor, theta_ctx: Tensor, x_query: Tensor, with_log_prob: bool,
                    eps: float) -> Tuple[Tensor, Optional[Tensor]]:
        """Dimension loop through the tabpfn surface (reference :128-169 / :202-241)."""
        joint = torch.cat([x_ctx, theta_ctx], dim=1)
        dx = x_ctx.shape[1]
        feats = x_query
        lp = torch.zeros(x_query.shape[0]) if with_log_prob else None
        for k in range(theta_ctx.shape[1]):
            self._model.fit(joint[:, : dx + k], joint[:, dx + k])
            pred = self._model.predict(feats, output_type="full", quantiles=[])
            draw = pred["criterion"].sample(pred["logits"])
            if with_log_prob:
                dev = pred["logits"].device
                step = -pred["criterion"](pred["logits"], draw.to(dev))
                step = torch.where(step == float("-inf"), torch.log(torch.tensor(eps, device=step.device)), step)
                lp = lp.to(step.device)
                lp += step
            feats = torch.cat([feats, draw[:, None].to(feats.device)], dim=1)
        return feats[:, dx:], lp

    def _ar(self, x_ctx: Tensor, theta_ctx: Tensor, x_query: Tensor, with_log_prob: bool,
            eps: float, row_base: int = 0, x_unique: Optional[Tensor] = None) -> Tuple[Tensor, Optional[Tensor]]:
        """``x_unique``: the distinct rows when ``x_query`` = ``x_unique.repeat_interleave(N // U, 0)``
        (the fused engine then runs AR step 0 once per distinct row)."""
        if self._fused():
            return self._model.ar_sample(x_ctx, theta_ctx, x_query, with_log_prob=with_log_prob, eps=eps,
                                         row_base=row_base, x_unique=x_unique)
        return self._ar_generic(x_ctx, theta_ctx, x_query, with_log_prob, eps)

    def _sample(self, sampling_batch_size: int, x: Tensor, repeat_x: bool = True, with_log_prob: bool = False,
                eps: float = 1e-15, row_base: int = 0, ar: Optional[Callable] = None) -> Tuple[Tensor, Optional[Tensor]]:
        """One batch of posterior draws for a single observation (reference :111-169).

        ``row_base``: Philox row of the batch's first draw (a row shard of a larger batch,
        npe_pfn.distributed); ``ar``: an alternative implementation of the dimension loop
        with :meth:`_ar`'s signature (the estimator-parallel multi-GPU loop).
        """
        x_query = x.repeat(sampling_batch_size, 1) if repeat_x else x
        x_unique = x if repeat_x and x.shape[0] == 1 else None  # one observation: every query row is x
        theta_ctx, x_ctx = self.get_context(x)
        if ar is not None:
            return ar(x_ctx, theta_ctx, x_query, with_log_prob, eps, row_base, x_unique=x_unique)
        return self._ar(x_ctx, theta_ctx, x_query, with_log_prob, eps, row_base=row_base, x_unique=x_unique)

    def _sample_batched(self, x: Tensor, num_samples_per_obs: int, with_log_prob: bool = False,
                        eps: float = 1e-15) -> Tuple[Tensor, Optional[Tensor]]:
        """Obs-major interleaved batch over all observations with the full context (reference :171-251)."""
        n_obs = x.shape[0]
        x_query = x.repeat_interleave(num_samples_per_obs, dim=0)
        # an observation shard [a, b) of a larger batch (npe_pfn.distributed) draws at the
        # Philox rows of the unsharded obs-major batch: row_base = a * samples per obs
        theta, lp = self._ar(self._x_train, self._theta_train, x_query, with_log_prob, eps,
                             row_base=self._obs_offset * num_samples_per_obs,
                             x_unique=x if num_samples_per_obs > 0 else None)
        theta = theta.reshape(n_obs, num_samples_per_obs, -1)
        if with_log_prob:
            return theta, lp.reshape(n_obs, num_samples_per_obs)
        return theta, None

    # ---------------------------------------------------------------- public
    def sample(self, sample_shape: torch.Size = torch.Size(), x: Tensor = None, max_sampling_batch_size: int = 10_000,
               with_log_prob: bool = False, eps: float = 1e-15, max_iter_rejection: Optional[int] = None,
               show_progress_bars: bool = False) -> Union[Tensor, Tuple[Tensor, Tensor]]:
        """Posterior draws for ONE observation with prior-support rejection (reference :253-308)."""
        return self._sample_impl(sample_shape, x, max_sampling_batch_size, with_log_prob, eps, max_iter_rejection)

    def _sample_impl(self, sample_shape, x, max_sampling_batch_size: int, with_log_prob: bool, eps: float,
                     max_iter_rejection: Optional[int], row_base_of: Optional[Callable[[int], int]] = None,
                     ar: Optional[Callable] = None):
        """``sample`` with two multi-GPU hooks (npe_pfn.distributed): ``row_base_of(i)`` = Philox
        row of the first draw of accept/reject batch i, ``ar`` = the dimension loop to use."""
        x = self._validate_x(self._embed(x) if self.embedding_net else x)
        if x.shape[0] > 1:
            raise ValueError(".sample() supports only `batchsize == 1`. If you intend to sample multiple "
                             "observations, use `.sample_batched()`. ")
        out_device = x.device
        batch_index = [0]

        def proposal(batch_size, **_):
            i = batch_index[0]
            batch_index[0] += 1
            rb = row_base_of(i) if row_base_of is not None else 0
            return self._sample(batch_size, x, repeat_x=True, with_log_prob=with_log_prob, eps=eps, row_base=rb,
                                ar=ar)

        with (self._reuse_fits() if ar is None else contextlib.nullcontext()):
            samples, log_probs, _ = accept_reject_sample(
                proposal=proposal,
                accept_reject_fn=self._within_support,
                num_samples=torch.Size(sample_shape).numel(),
                show_progress_bars=self.show_progress_bars,
                max_sampling_batch_size=max_sampling_batch_size,
                proposal_sampling_kwargs={},
                max_iter_rejection=max_iter_rejection,
            )
        samples = samples.to(out_device)
        if with_log_prob:
            return samples, log_probs.to(out_device)
        return samples

    def sample_batched(self, x: Tensor, sample_shape: torch.Size = torch.Size(), max_sampling_batch_size: int = 10_000,
                       with_log_prob: bool = False, eps: float = 1e-15, oversample_factor: float = 1.5,
                       show_progress_bars: bool = False) -> Union[Tensor, Tuple[Tensor, Tensor]]:
        """Posterior draws for many observations at once (reference :310-410).

        ``max_sampling_batch_size`` is accepted and, as in the reference, not used.
        """
        x = self._validate_x(self._embed(x) if self.embedding_net else x)
        n_obs = x.shape[0]
        n = torch.Size(sample_shape).numel()
        if self.prior is None:
            th, lp = self._sample_batched(x, n, with_log_prob=with_log_prob, eps=eps)
            th = th.to(x.device)
            return (th, lp.to(x.device)) if with_log_prob else th
        # Per-observation rejection (reference :360-397), vectorised over observations on the
        # samples' device: an accepted draw's rank within its observation decides whether it is
        # taken and where it lands, so every observation keeps its first accepted draws in
        # order, as the reference's per-observation loop does, with one host sync per round.
        per_round = int(n * oversample_factor)
        with self._reuse_fits():
            return self._sample_batched_rounds(x, n, n_obs, per_round, with_log_prob, eps)

    def _sample_batched_rounds(self, x, n, n_obs, per_round, with_log_prob, eps):
        out_th = out_lp = None
        need = filled = None
        for _ in range(10):
            if need is not None and int(need.sum()) == 0:
                break
            th, lp = self._sample_batched(x, per_round, with_log_prob=with_log_prob, eps=eps)
            dev = th.device
            if out_th is None:
                out_th = torch.empty(n_obs, n, th.shape[-1], dtype=th.dtype, device=dev)
                out_lp = torch.empty(n_obs, n, dtype=lp.dtype, device=dev) if with_log_prob else None
                need = torch.full((n_obs,), n, dtype=torch.int64, device=dev)
                filled = torch.zeros(n_obs, dtype=torch.int64, device=dev)
            ok = self._within_support(th.reshape(n_obs * per_round, -1)).reshape(n_obs, per_round).to(dev)
            rank = torch.cumsum(ok.to(torch.int64), 1) - 1
            sel = ok & (rank < need[:, None])
            oi, ri = sel.nonzero(as_tuple=True)
            dest = filled[oi] + rank[oi, ri]
            out_th[oi, dest] = th[oi, ri]
            if with_log_prob:
                out_lp[oi, dest] = lp.to(dev)[oi, ri]
            taken = sel.sum(1)
            filled += taken
            need -= taken
        if int(need.sum()) != 0:
            # the reference's final torch.stack fails on unequal per-observation counts
            raise RuntimeError(f"sample_batched: {int((need > 0).sum())} observation(s) got fewer than {n} "
                               f"samples inside the prior support after 10 rounds")
        samples = out_th.to(x.device)
        if with_log_prob:
            return samples, out_lp.to(x.device)
        return samples

    def log_prob(self, theta: Tensor, x: Tensor, max_sampling_batch_size: int = 10_000, mode: str = "autoregressive",
                 eps: float = 1e-15, **ratio_kwargs) -> Tensor:
        """log q(theta | x), in chunks of ``max_sampling_batch_size`` rows (reference :412-455)."""
        if self.embedding_net:
            x = self._embed(x)
        theta = self._validate_theta(theta)
        x = self._validate_x(x)
        if mode not in ("autoregressive", "ratio_based"):
            raise ValueError(f"Invalid mode: {mode}")
        out = torch.zeros(theta.shape[0])
        with (self._reuse_fits() if mode == "autoregressive" else contextlib.nullcontext()):
            for i in range(0, theta.shape[0], max_sampling_batch_size):
                chunk = theta[i: i + max_sampling_batch_size]
                if mode == "autoregressive":
                    out[i: i + max_sampling_batch_size] = self._autoregressive_log_prob(chunk, x, eps=eps).cpu()
                else:
                    out[i: i + max_sampling_batch_size] = self._ratio_based_log_prob(chunk, x, eps=eps,
                                                                                     **ratio_kwargs).cpu()
        return out

    def log_prob_batched(self, theta: Tensor, x: Tensor):
        raise NotImplementedError

    def _autoregressive_log_prob(self, theta: Tensor, x: Tensor = None, repeat_x: bool = True,
                                 eps: float = 1e-15) -> Tensor:
        """Teacher-forced sum of per-dimension log densities (reference :462-524)."""
        n = theta.shape[0]
        x_query = x.repeat(n, 1) if repeat_x else x
        assert x_query.shape[0] == n
        theta_ctx, x_ctx = self.get_context(x)
        if hasattr(self._model, "ar_log_prob"):
            x_unique = x if repeat_x and x.shape[0] == 1 else None  # one observation: every query row is x
            return self._model.ar_log_prob(x_ctx, theta_ctx, x_query, theta, eps=eps, x_unique=x_unique)
        joint = torch.cat([x_ctx, theta_ctx], dim=1)
        test = torch.cat([x_query, theta], dim=1)
        dx = x_ctx.shape[1]
        lp = torch.zeros(n)
        for k in range(theta_ctx.shape[1]):
            self._model.fit(joint[:, : dx + k], joint[:, dx + k])
            pred = self._model.predict(test[:, : dx + k], output_type="full", quantiles=[])
            step = -pred["criterion"](pred["logits"], test[:, dx + k])
            step = torch.where(step == float("-inf"), torch.log(torch.tensor(eps)), step)
            lp += step
        return lp

    def _ratio_based_log_prob(self, theta: Tensor, x: Tensor = None, num_posterior_samples: int = 5000,
                              boundary_padding: float = 0.1, reuse_estimator_if_possible: bool = True,
                              eps: float = 1e-15) -> Tensor:
        """Classifier-based density ratio (reference :526-570) -- needs the classifier engine."""
        if self._model_classifier is None:
            self._model_classifier = DensityRatioWrapper(**self.classifier_init_kwargs)
        theta_ctx, x_ctx = self.get_context(x)
        if not reuse_estimator_if_possible or self._model_classifier.refit_necessary(
                x, x_ctx, theta_ctx, num_posterior_samples, boundary_padding):
            post = self.sample(sample_shape=torch.Size([num_posterior_samples]), x=x)
            self._model_classifier.fit(x, post, boundary_padding, x_ctx, theta_ctx)
        return self._model_classifier.ratio_log_probs(theta, eps)

    def _get_classifier_bounds(self):
        if self._model_classifier is None:
            return None, None
        return self._model_classifier._padded_dim_min, self._model_classifier._padded_dim_max

    def _within_support(self, theta: Tensor) -> Tensor:
        """Prior-support mask (reference :581-600).

        On the GPU a box prior (BoxUniform / Independent(Uniform)) is checked by
        the K9 kernel ``npfn_box_support``; any other prior is evaluated by torch
        on the prior's own device.
        """
        if theta.is_cuda and self._fused():
            bounds = _box_bounds(self.prior)
            if bounds is not None:
                return self._model.engine.box_support(theta, bounds[0], bounds[1])
        try:
            return self._support_mask(theta).to(theta.device)
        except RuntimeError:
            # parameters of the prior live on another device (e.g. a CPU box prior)
            prior_dev = _distribution_device(self.prior)
            return self._support_mask(theta.to(prior_dev)).to(theta.device)

    def _support_mask(self, th: Tensor) -> Tensor:
        try:
            chk = self.prior.support.check(th)
            if chk.shape == th.shape:
                chk = torch.all(chk, dim=-1)
            return chk
        except (NotImplementedError, AttributeError):
            return torch.isfinite(self.prior.log_prob(th))


def _distribution_device(dist) -> Optional[torch.device]:
    base = dist
    while hasattr(base, "base_dist"):
        base = base.base_dist
    for name in ("loc", "low", "scale", "high", "probs", "logits", "covariance_matrix"):
        t = getattr(base, name, None)
        if isinstance(t, Tensor):
            return t.device
    return None


def _box_bounds(prior) -> Optional[Tuple[Tensor, Tensor]]:
    """(low, high) if the prior is a box uniform, else None."""
    base = prior
    if isinstance(base, torch.distributions.Independent):
        base = base.base_dist
    if isinstance(base, torch.distributions.Uniform):
        return base.low.reshape(-1), base.high.reshape(-1)
    return None


class DensityRatioWrapper:
    """Ratio-based log density q(θ|x) ∝ U_box(θ) · p(post|θ) / p(unif|θ) (reference :603-704).

    ``fit`` draws as many uniform samples on the padded bounding box of the
    posterior samples as there are posterior samples and trains the engine
    classifier (``TabPFNClassifier``, label 0 = uniform, 1 = posterior);
    ``ratio_log_probs`` = log U + log(p1 + eps) - log(p0 + eps) inside the box and
    log U + log eps - log(1 + eps) outside it.  The classifier is reused while
    x, the context and the settings are unchanged (``refit_necessary``).  All
    tensors stay on the device of the posterior samples.
    """

    def __init__(self, **init_kwargs):
        self._classifier = TabPFNClassifier(**init_kwargs)
        self._ratio_log_prob_x = None
        self._num_posterior_samples = None
        self._boundary_padding = None
        self._padded_dim_min = None
        self._padded_dim_max = None
        self._uniform_log_prob = None

    def fit(self, x: Tensor, posterior_samples: Tensor, boundary_padding: float, x_context: Tensor,
            theta_context: Tensor) -> None:
        lo = posterior_samples.min(dim=0).values
        hi = posterior_samples.max(dim=0).values
        span = hi - lo
        pad_lo = lo - boundary_padding * span
        pad_hi = hi + boundary_padding * span
        pad_span = pad_hi - pad_lo
        uniform_log_prob = -torch.log(pad_span).sum()
        uniform = torch.rand_like(posterior_samples) * pad_span + pad_lo
        n = posterior_samples.shape[0]
        X = torch.cat([uniform, posterior_samples], dim=0)
        y = torch.cat([torch.zeros(n), torch.ones(n)], dim=0)
        self._ratio_log_prob_x = x
        self._num_posterior_samples = n
        self._boundary_padding = boundary_padding
        self._x_context = x_context
        self._theta_context = theta_context
        self._padded_dim_min = pad_lo
        self._padded_dim_max = pad_hi
        self._uniform_log_prob = uniform_log_prob
        self._classifier.fit(X, y)

    def refit_necessary(self, x: Tensor, x_context: Tensor, theta_context: Tensor, num_posterior_samples: int,
                        boundary_padding: float) -> bool:
        if self._ratio_log_prob_x is None:
            return True
        return not (torch.allclose(x, self._ratio_log_prob_x)
                    and x_context.shape == self._x_context.shape and torch.allclose(x_context, self._x_context)
                    and theta_context.shape == self._theta_context.shape
                    and torch.allclose(theta_context, self._theta_context)
                    and num_posterior_samples == self._num_posterior_samples
                    and math.isclose(boundary_padding, self._boundary_padding))

    def _proba(self, theta: Tensor) -> Tensor:
        clf = self._classifier
        if hasattr(clf, "predict_proba_tensor"):
            return clf.predict_proba_tensor(theta).to(theta.device)
        return torch.as_tensor(clf.predict_proba(theta)).to(theta.device)  # numpy, as tabpfn returns it

    def ratio_log_probs(self, theta: Tensor, eps: float = 1e-15) -> Tensor:
        lo = self._padded_dim_min.to(theta.device)
        hi = self._padded_dim_max.to(theta.device)
        inside = torch.all((theta >= lo) & (theta <= hi), dim=1)
        ulp = self._uniform_log_prob.to(theta.device)
        outside_val = ulp + torch.log(torch.tensor(eps)).to(theta.device) - torch.log(torch.tensor(1 + eps)).to(theta.device)
        out = outside_val.expand(theta.shape[0]).clone()
        if inside.any():
            p = self._proba(theta[inside])
            out[inside] = ulp + torch.log(p[:, 1] + eps) - torch.log(p[:, 0] + eps)
        return out


class TabPFN_Based_NPE_PFN(NPE_PFN_Core):
    """NPE-PFN whose context is filtered per observation (reference :708-744)."""

    def __init__(
        self,
        show_progress_bars: bool = False,
        prior: Optional[Distribution] = None,
        filter_type: Union[str, Callable] = "standardized_euclidean_filtering",
        filter_context_size: int = 10_000,
        regressor_init_kwargs: Mapping = {},
        classifier_init_kwargs: Mapping = {},
        embedding_net: Optional[torch.nn.Module] = None,
        x_shape: Optional[torch.Size] = None,
    ):
        super().__init__(show_progress_bars, prior, regressor_init_kwargs=regressor_init_kwargs,
                         classifier_init_kwargs=classifier_init_kwargs, embedding_net=embedding_net,
                         x_shape=x_shape)
        self.filter = get_filtering_method(filter_type)
        self.filter_context_size = filter_context_size

    def _context_is_deterministic(self) -> bool:
        # random_filtering draws a new randperm subset per call; a user callable is unknown
        return self.filter in DETERMINISTIC_FILTERS

    def get_context(self, x: Tensor) -> Tuple[Tensor, Tensor]:
        x = self._validate_x(x)
        return self.filter(x, self._theta_train, self._x_train, self.filter_context_size)
