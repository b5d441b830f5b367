"""Deterministic synthetic tabular data generated directly in device memory.

Features are quantized to ``levels`` distinct values per column (default
256; ``levels=None`` gives continuous N(0, 1) features, for the exact
presorted-list engine). Labels come from a random linear score plus a
sparse interaction term and Gaussian noise, which makes trees grow deep and
wide like on real tabular data.
"""

from __future__ import annotations

import torch

__all__ = ["make_classification", "make_regression"]


def _features(n, F, levels, gen, device, dtype):
    if levels is None:  # continuous: every value distinct (exact-threshold engine)
        return torch.randn((n, F), generator=gen, device=device, dtype=dtype)
    X = torch.randint(0, levels, (n, F), generator=gen, device=device, dtype=torch.int32)
    return X.to(dtype)


def _score(X, gen, device, noise, levels):
    n, F = X.shape
    w = torch.randn(F, generator=gen, device=device)
    Xc = X.float() * 0.25 if levels is None else X.float() / max(levels - 1, 1) - 0.5
    s = Xc @ w
    k = min(F, 8)
    s = s + 2.0 * (Xc[:, :k:2] * Xc[:, 1:k:2]).sum(1) if k >= 2 else s
    s = s / (s.std() + 1e-12)
    return s + noise * torch.randn(n, generator=gen, device=device)


def make_classification(n, F, *, n_classes=2, levels=256, noise=0.3, seed=0, device="cuda",
                        dtype=torch.float32):
    """Return ``(X [n,F], y [n] int64)`` on ``device``."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    X = _features(n, F, levels, gen, device, dtype)
    s = _score(X, gen, device, noise, levels)
    qs = torch.quantile(s[: min(n, 1 << 20)].float(),
                        torch.linspace(0, 1, n_classes + 1, device=device)[1:-1])
    y = torch.bucketize(s, qs).to(torch.int64)
    return X, y


def make_regression(n, F, *, levels=256, noise=0.3, seed=0, device="cuda", dtype=torch.float32):
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    X = _features(n, F, levels, gen, device, dtype)
    y = _score(X, gen, device, noise, levels).double()
    return X, y
