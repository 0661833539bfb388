"""Truncated sequential NPE-PFN (reference: npe_pfn/tsnpe_pfn.py:14-119).

Round loop: draw simulations from the current proposal, append ALL rounds'
simulations as context, and build a :class:`PosteriorSupport` that becomes the
next proposal.  ``sbi.inference.simulate_for_sbi`` (sbi 0.23.3, absent here)
is replaced by :func:`simulate`, which draws ``theta`` from the proposal and
calls the simulator in batches.
"""

from __future__ import annotations

import logging
from typing import Callable, Mapping

import torch
from torch.distributions import Distribution

from .npe_pfn import TabPFN_Based_NPE_PFN
from .support_posterior import PosteriorSupport

log = logging.getLogger(__name__)


def simulate(simulator: Callable, proposal, num_simulations: int, simulation_batch_size: int = 1000):
    theta = proposal.sample((num_simulations,))
    xs = [simulator(theta[i: i + simulation_batch_size]) for i in range(0, num_simulations, simulation_batch_size)]
    return theta, torch.cat(xs, dim=0)


def run_tsnpe_pfn(
    simulator: Callable,
    prior: Distribution,
    observation: torch.Tensor,
    num_simulations: int = 10_000,
    num_rounds: int = 10,
    proposal_batch_size: int = 1000,
    simulation_batch_size: int = 1000,
    num_samples_to_estimate_support: int = 10_000,
    allowed_false_negatives: float = 0.0001,
    context_size: int = 10_000,
    log_prob_mode: str = "ratio_based",
    sampling_method: str = "rejection",
    max_iter_rejection: int = 1000,
    oversample_sir: int = 100,
    filtering: str = "no_filtering",
    regressor_init_kwargs: Mapping = {},
    classifier_init_kwargs: Mapping = {},
):
    """Runs TSNPE-PFN and returns the final ``TabPFN_Based_NPE_PFN``."""
    per_round = num_simulations if num_rounds == 1 else num_simulations // num_rounds
    log.info(f"Running {'NPE_PFN' if num_rounds == 1 else 'TSNPE_PFN'}; {per_round} simulations per round")
    if simulation_batch_size > per_round:
        simulation_batch_size = per_round
        log.warning("Reduced simulation_batch_size to num_simulation_per_round")
    estimator = TabPFN_Based_NPE_PFN(prior=prior, regressor_init_kwargs=regressor_init_kwargs,
                                     classifier_init_kwargs=classifier_init_kwargs, filter_type=filtering,
                                     filter_context_size=context_size)
    proposal = prior
    thetas, xs = [], []
    posterior = estimator
    for r in range(num_rounds):
        log.info(f"Round {r + 1}/{num_rounds}")
        theta, x = simulate(simulator, proposal, per_round, simulation_batch_size)
        thetas.append(theta)
        xs.append(x)
        posterior = estimator.append_simulations(torch.cat(thetas, 0), torch.cat(xs, 0))
        if r == num_rounds - 1:
            break
        proposal = PosteriorSupport(
            prior, posterior, obs=observation,
            num_samples_to_estimate_support=num_samples_to_estimate_support,
            batch_size_for_estimate_support=proposal_batch_size,
            allowed_false_negatives=allowed_false_negatives,
            sampling_method=sampling_method,
            max_iter_rejection=max_iter_rejection,
            oversample_sir=oversample_sir,
            log_prob_kwargs={"mode": log_prob_mode},
        )
    return posterior
