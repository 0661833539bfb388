"""Classifier two-sample test (C2ST), restated from the reference's evaluation harness.

Follows ``classifier_two_samples_test_torch`` in scripts/evaluate_ropefm.py:119-280 of
the reference: z-score both sets by the first set's mean / unbiased std (:165-170), label
X 0 and Y 1, StratifiedKFold(5, shuffle, random_state=seed) (:196-199), per fold the
``DefaultMLP`` (:60-80: dim -> 4d -> 8d -> 8d -> 4d -> 2, ReLU) trained with Adam
(lr 1e-3, batch 128, 100 epochs, cross-entropy), score = mean held-out accuracy.
0.5 = indistinguishable.  Test infrastructure only; runs on the CPU.
"""
from __future__ import annotations

import numpy as np
import torch
from sklearn.model_selection import StratifiedKFold


def _mlp(d: int) -> torch.nn.Module:
    h = 8 * d
    return torch.nn.Sequential(
        torch.nn.Linear(d, h // 2), torch.nn.ReLU(),
        torch.nn.Linear(h // 2, h), torch.nn.ReLU(),
        torch.nn.Linear(h, h), torch.nn.ReLU(),
        torch.nn.Linear(h, h // 2), torch.nn.ReLU(),
        torch.nn.Linear(h // 2, 2),
    )


def c2st(X, Y, seed: int = 1, n_folds: int = 5, epochs: int = 100, batch_size: int = 128,
         lr: float = 1e-3) -> float:
    X = torch.as_tensor(np.asarray(X), dtype=torch.float32)
    Y = torch.as_tensor(np.asarray(Y), dtype=torch.float32)
    g = torch.Generator().manual_seed(seed)
    mu, sd = X.mean(0), X.std(0)
    sd = torch.where(sd == 0, torch.ones_like(sd), sd)
    X, Y = (X - mu) / sd, (Y - mu) / sd
    data = torch.cat([X, Y]).numpy()
    labels = np.concatenate([np.zeros(len(X), dtype=np.int64), np.ones(len(Y), dtype=np.int64)])
    scores = []
    for tr, te in StratifiedKFold(n_splits=n_folds, shuffle=True, random_state=seed).split(data, labels):
        torch.manual_seed(seed)
        net = _mlp(data.shape[1])
        opt = torch.optim.Adam(net.parameters(), lr=lr)
        xt, yt = torch.from_numpy(data[tr]), torch.from_numpy(labels[tr])
        net.train()
        for _ in range(epochs):
            perm = torch.randperm(len(xt), generator=g)
            for i in range(0, len(xt), batch_size):
                idx = perm[i:i + batch_size]
                opt.zero_grad()
                loss = torch.nn.functional.cross_entropy(net(xt[idx]), yt[idx])
                loss.backward()
                opt.step()
        net.eval()
        with torch.no_grad():
            pred = net(torch.from_numpy(data[te])).argmax(1).numpy()
        scores.append(float((pred == labels[te]).mean()))
    return float(np.mean(scores))
