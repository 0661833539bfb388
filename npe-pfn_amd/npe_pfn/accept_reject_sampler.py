"""Rejection loop around a batch proposal (reference: npe_pfn/accept_reject_sampler.py:9-91).

Behaviour kept from the reference (pinned by tests/golden/accrej.npz):

* the first batch is ``min(num_samples, max_sampling_batch_size)``;
* after every batch the next size is
  ``min(max_bs, max(int(1.5 * remaining / max(rate, 1e-12)), 100))`` with
  ``rate`` = accepted so far / proposed so far (reference :68-72);
* after ``max_iter_rejection`` iterations the last batch is appended unfiltered
  (reference :74-77);
* the result is trimmed to ``num_samples`` and returned as a 3-tuple
  ``(samples, log_probs or None, acceptance_rate)`` (reference :82-91).

Candidates may live on the GPU: the mask and the compaction stay on the
candidates' device, so the fused sampler's output never leaves HBM here.
"""

from __future__ import annotations

from typing import Callable, Dict, Optional, Tuple

import torch
from torch import Tensor
from tqdm import tqdm


@torch.no_grad()
def accept_reject_sample(
    proposal: Callable,
    accept_reject_fn: Callable,
    num_samples: int,
    show_progress_bars: bool = False,
    max_sampling_batch_size: int = 10_000,
    proposal_sampling_kwargs: Optional[Dict] = None,
    max_iter_rejection: Optional[int] = None,
) -> Tuple[Tensor, Optional[Tensor], float]:
    kwargs = proposal_sampling_kwargs or {}
    bar = tqdm(disable=not show_progress_bars, total=num_samples,
               desc=f"Drawing {num_samples} posterior samples")
    kept, kept_lp = [], []
    n_kept = 0
    n_proposed = 0
    remaining = num_samples
    batch = min(num_samples, max_sampling_batch_size)
    iteration = 0
    while remaining > 0:
        iteration += 1
        candidates, log_probs = proposal(batch, **kwargs)
        mask = accept_reject_fn(candidates)
        if mask.device != candidates.device:
            mask = mask.to(candidates.device)
        kept.append(candidates[mask])
        if log_probs is not None:
            kept_lp.append(log_probs[mask])
        n_acc = int(kept[-1].shape[0])
        n_kept += n_acc
        n_proposed += batch
        remaining -= n_acc
        bar.update(n_acc)
        rate = n_kept / n_proposed
        batch = min(max_sampling_batch_size, max(int(1.5 * remaining / max(rate, 1e-12)), 100))
        if max_iter_rejection is not None and iteration > max_iter_rejection:
            kept.append(candidates)
            if log_probs is not None:
                kept_lp.append(log_probs)
            break
    bar.close()
    samples = torch.cat(kept, dim=0)[:num_samples]
    lps = torch.cat(kept_lp, dim=0)[:num_samples] if kept_lp else None
    return samples, lps, len(samples) / n_proposed
