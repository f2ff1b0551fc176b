"""Seeded synthetic MRI/PET embedding pairs.

iid Gaussian embeddings make Sinkhorn converge trivially, so the benchmark and
the parity fixtures use *paired, structured* embeddings instead:

    Z ~ N(0, 1)^{N x r}            shared latent per subject (r = 32)
    label ~ Bernoulli(0.5)         AD / CN analogue
    mu_c ~ 0.5 * N(0, 1)^d         class centroids, c in {0, 1}
    X = relu(Z A + mu_label + 0.1 xi)     "MRI" embedding   (A ~ N(0, 1/r)^{r x d})
    Y = relu(Z B + mu_label + 0.1 xi')    "PET" embedding   (B ~ N(0, 1/r)^{r x d})

All draws come from ``numpy.random.default_rng(seed)`` in a fixed order, so a
seed pins the arrays bit for bit on every machine.
"""
from __future__ import annotations

import numpy as np


def paired_embeddings(n: int, d: int, seed: int = 1234, r: int = 32, d2: int | None = None):
    """Return ``(X, Y, labels)``: float32 ``(n, d)``, float32 ``(n, d2)``, int64 ``(n,)``."""
    d2 = d if d2 is None else d2
    rng = np.random.default_rng(seed)
    z = rng.standard_normal((n, r))
    labels = (rng.random(n) < 0.5).astype(np.int64)
    mu_x = 0.5 * rng.standard_normal((2, d))
    mu_y = 0.5 * rng.standard_normal((2, d2))
    a = rng.standard_normal((r, d)) / np.sqrt(r)
    b = rng.standard_normal((r, d2)) / np.sqrt(r)
    x = np.maximum(z @ a + mu_x[labels] + 0.1 * rng.standard_normal((n, d)), 0.0)
    y = np.maximum(z @ b + mu_y[labels] + 0.1 * rng.standard_normal((n, d2)), 0.0)
    return x.astype(np.float32), y.astype(np.float32), labels


def uniform(n: int) -> np.ndarray:
    """``ot.unif(n)``: the uniform histogram used for a and b (MRI_PET_OT_nojax.py:139-140)."""
    return np.full(n, 1.0 / n, dtype=np.float64)
