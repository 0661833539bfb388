"""Simulators and priors of the benchmark configurations (BASELINE.json configs c1-c5).

* Gaussian-linear (sbibm ``gaussian_linear``): theta ~ N(0, 0.1 I_D),
  x = theta + sqrt(0.1) eps -- c1, c2, c5;
* SLCP (sbibm ``slcp``): theta ~ U(-3, 3)^5, four iid 2-D points from
  N((theta_1, theta_2), S) with s_1 = theta_3^2, s_2 = theta_4^2,
  rho = tanh(theta_5) -- c3;
* two moons as in the reference demo (demo.ipynb cell 2), prior U(-1, 1)^2,
  theta_o = 0.5 * 1 -- c4.

Inputs for the bench and the tests; not on the sampling hot path.
"""

from __future__ import annotations

import math

import numpy as np
import torch
from torch.distributions import Independent, Normal, Uniform

__all__ = ["gaussian_linear_prior", "gaussian_linear", "gaussian_linear_task", "slcp_prior", "slcp_simulator",
           "slcp_task", "two_moons_prior", "two_moons_simulator"]


def gaussian_linear_prior(D: int, device="cpu") -> Independent:
    return Independent(Normal(torch.zeros(D, device=device), torch.full((D,), math.sqrt(0.1), device=device)), 1)


def gaussian_linear(theta: torch.Tensor, generator=None) -> torch.Tensor:
    return theta + torch.randn(theta.shape, generator=generator, device=theta.device) * math.sqrt(0.1)


def gaussian_linear_task(D: int, n: int, seed: int = 0):
    """(theta [n, D], x [n, D], x_o [1, D]) with x_o simulated from theta_o ~ prior (seeds seed, seed + 1)."""
    g = torch.Generator().manual_seed(seed)
    theta = torch.randn(n, D, generator=g) * math.sqrt(0.1)
    x = theta + torch.randn(n, D, generator=g) * math.sqrt(0.1)
    g1 = torch.Generator().manual_seed(seed + 1)
    theta_o = torch.randn(1, D, generator=g1) * math.sqrt(0.1)
    x_o = theta_o + torch.randn(1, D, generator=g1) * math.sqrt(0.1)
    return theta.float(), x.float(), x_o.float()


def slcp_prior(device="cpu") -> Independent:
    return Independent(Uniform(torch.full((5,), -3.0, device=device), torch.full((5,), 3.0, device=device)), 1)


def slcp_simulator(theta: torch.Tensor, generator=None) -> torch.Tensor:
    """sbibm SLCP: x = 4 points ~ N(m, S), m = theta[:2], S from (theta_3^2, theta_4^2, tanh theta_5)."""
    m = theta[:, :2]
    s1, s2 = theta[:, 2] ** 2, theta[:, 3] ** 2
    rho = torch.tanh(theta[:, 4])
    z = torch.randn((theta.shape[0], 4, 2), generator=generator, device=theta.device)
    # Cholesky of [[s1^2, rho s1 s2], [rho s1 s2, s2^2]]
    x0 = s1[:, None] * z[..., 0]
    x1 = s2[:, None] * (rho[:, None] * z[..., 0] + torch.sqrt(1 - rho[:, None] ** 2) * z[..., 1])
    pts = torch.stack([x0, x1], -1) + m[:, None, :]
    return pts.reshape(theta.shape[0], 8)


def slcp_task(n: int, seed: int = 0):
    g = torch.Generator().manual_seed(seed)
    theta = torch.rand(n, 5, generator=g) * 6 - 3
    x = slcp_simulator(theta, g)
    g1 = torch.Generator().manual_seed(seed + 1)
    theta_o = torch.rand(1, 5, generator=g1) * 6 - 3
    return theta.float(), x.float(), slcp_simulator(theta_o, g1).float()


def two_moons_prior() -> Uniform:
    """The demo's prior: a plain ``Uniform(-1, 1)`` over 2 dims (not Independent, demo.ipynb:78)."""
    return Uniform(-torch.ones(2), torch.ones(2))


def two_moons_simulator(theta: torch.Tensor) -> torch.Tensor:
    """Two-moons simulator of the reference demo (demo.ipynb:50-75), global torch RNG."""
    n = theta.shape[0]
    a = Uniform(torch.full((n,), -np.pi / 2), torch.full((n,), np.pi / 2)).rsample()
    r = Normal(torch.full((n,), 0.1), torch.full((n,), 0.01)).rsample()
    p = torch.stack([r * torch.cos(a) + 0.25, r * torch.sin(a)], 1)
    th = theta.cpu()
    q = torch.stack([-torch.abs(th[:, 0] + th[:, 1]) / np.sqrt(2), (-th[:, 0] + th[:, 1]) / np.sqrt(2)], 1)
    return (p + q).to(theta.device)
