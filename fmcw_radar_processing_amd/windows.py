"""Window taps of the MATLAB host (radar_processing.m:138, :139, :276).

These are the product host's own implementations of MATLAB's documented
window definitions (symmetric forms, computed on one half and mirrored the
way MATLAB's ``gencoswin`` / ``chebwin`` / ``kaiser`` do).  The test oracle
uses scipy.signal.windows as an independent implementation.
"""
from __future__ import annotations

import numpy as np


def _mirror(half: np.ndarray, n: int) -> np.ndarray:
    return np.concatenate([half, half[::-1]]) if n % 2 == 0 else np.concatenate([half, half[-2::-1]])


def blackman(n: int) -> np.ndarray:
    """blackman(n) ('symmetric'): 0.42 - 0.5 cos(2 pi x) + 0.08 cos(4 pi x), x = k/(n-1)."""
    if n == 1:
        return np.ones(1)
    m = n // 2 if n % 2 == 0 else (n + 1) // 2
    x = np.arange(m) / (n - 1)
    w = 0.42 - 0.5 * np.cos(2 * np.pi * x) + 0.08 * np.cos(4 * np.pi * x)
    w[0] = 0.0  # exact zero end points (0.42 - 0.5 + 0.08 rounds to -1.4e-17)
    return _mirror(w, n)


def hann(n: int) -> np.ndarray:
    """hann(n) ('symmetric'): 0.5 (1 - cos(2 pi k/(n-1)))."""
    if n == 1:
        return np.ones(1)
    m = n // 2 if n % 2 == 0 else (n + 1) // 2
    x = np.arange(m) / (n - 1)
    return _mirror(0.5 - 0.5 * np.cos(2 * np.pi * x), n)


def kaiser(n: int, beta: float) -> np.ndarray:
    """kaiser(n, beta) = I0(beta sqrt(1 - (2k/(n-1) - 1)^2)) / I0(beta)."""
    if n == 1:
        return np.ones(1)
    k = np.arange(n)
    r = 2.0 * k / (n - 1) - 1.0
    return np.i0(beta * np.sqrt(np.clip(1.0 - r * r, 0.0, None))) / np.i0(beta)


def chebwin(n: int, r: float = 100.0) -> np.ndarray:
    """chebwin(n, r) (Dolph-Chebyshev, r dB sidelobes; MATLAB default r = 100).

    Evaluate the Chebyshev polynomial T_{n-1}(beta cos(pi k / n)) on the unit
    circle and take its DFT (with the half-sample shift for even n), then
    normalise the peak to 1.
    """
    if n == 1:
        return np.ones(1)
    order = n - 1.0
    beta = np.cosh(np.arccosh(10.0 ** (abs(r) / 20.0)) / order)
    k = np.arange(n)
    x = beta * np.cos(np.pi * k / n)
    p = np.empty(n)
    big, small, mid = x > 1, x < -1, np.abs(x) <= 1
    p[big] = np.cosh(order * np.arccosh(x[big]))
    p[small] = (2 * (n % 2) - 1) * np.cosh(order * np.arccosh(-x[small]))
    p[mid] = np.cos(order * np.arccos(x[mid]))
    if n % 2:
        w = np.real(np.fft.fft(p))
        h = (n + 1) // 2
        w = w[:h]
        w = np.concatenate([w[h - 1:0:-1], w])
    else:
        p = p * np.exp(1j * np.pi / n * k)
        w = np.real(np.fft.fft(p))
        h = n // 2 + 1
        w = np.concatenate([w[h - 1:0:-1], w[1:h]])
    return w / w.max()
