"""TEST INFRASTRUCTURE (checker only; never imported by the product path).

numpy restatement of the spectrogram picture of radar-etl-pipeline/
radar_processing.m:331-348 (surf of the fftshift-ed one-sided psd, view(0,90),
axis tight, ylim([0 150]), clim([-40 0]), colormap(jet), exportgraphics), with
the same rules the GPU renderer states (fmcw_radar_processing_amd/csrc/
kernels_render.hip) in the same float64 operation order, so that the indices
agree exactly given the same P.  MATLAB graphics cannot run here: these rules
are our reading of surf/flat shading/the depth test of the top view, so the
picture is parity-unpinned against MATLAB itself.
"""
from __future__ import annotations

import numpy as np


def jet(m: int = 256) -> np.ndarray:
    """MATLAB jet(m) (jet.m: n = ceil(m/4), u = [(1:n)/n ones(1,n-1) (n:-1:1)/n])."""
    n = -(-m // 4)
    u = np.concatenate([np.arange(1, n + 1) / n, np.ones(n - 1), np.arange(n, 0, -1) / n])
    g = (-(-n // 2)) - (1 if m % 4 == 1 else 0) + np.arange(1, len(u) + 1)
    r, b = g + n, g - n
    J = np.zeros((m, 3))
    gk, rk, bk = g[g <= m], r[r <= m], b[b >= 1]
    J[gk - 1, 1] = u[:len(gk)]
    J[rk - 1, 0] = u[:len(rk)]
    J[bk - 1, 2] = u[len(u) - len(bk):]
    return J


def jet_palette_u8() -> np.ndarray:
    return np.floor(jet(256) * 255.0 + 0.5).astype(np.uint8)   # lround of non-negative values


def render_indices(Q: np.ndarray, nq: int, pmax: float, nfft: int, fs: float, t0: float, dt: float,
                   W: int, H: int, fmax: float = 150.0, cmin: float = -40.0, cmax: float = 0.0) -> np.ndarray:
    """Palette indices [H][W] from Q[nseg][nq + 1] (P of bins 0..nq-1, then bin nfft/2)."""
    Q = np.asarray(Q, np.float64)
    nseg = Q.shape[0]
    nb = nfft // 2 + 1
    seam = nb - nb // 2 - 1
    out = np.zeros((H, W), np.uint8)
    if nseg < 2:
        return out
    inv = 1.0 / float(np.float32(pmax)) if pmax > 0 else 0.0
    with np.errstate(divide="ignore"):
        Z = np.where(Q > 0, 20.0 * np.log10(Q * inv), -1.0e30)
    Z = np.maximum(Z, -1.0e30)
    px = np.arange(W, dtype=np.float64)
    py = np.arange(H, dtype=np.float64)
    t1 = t0 + (nseg - 1) * dt
    t = t0 + (px + 0.5) * (t1 - t0) / W
    u = (t - t0) / dt
    s = np.clip(np.floor(u).astype(np.int64), 0, nseg - 2)
    fx = u - s
    y = fmax * (1.0 - (py + 0.5) / H)
    df, nyq_f = fs / nfft, fs * 0.5

    def bil(z00, z10, z01, z11, fy, fxx):
        a = z00 + (z10 - z00) * fy
        b = z01 + (z11 - z01) * fy
        return a + (b - a) * fxx

    S = np.broadcast_to(s[None, :], (H, W))
    FX = np.broadcast_to(fx[None, :], (H, W))
    Y = np.broadcast_to(y[:, None], (H, W))
    zf = bil(Z[S, 0], Z[S, nq], Z[S + 1, 0], Z[S + 1, nq], Y / nyq_f, FX)
    zc = Z[S, nq].copy()
    my = Y / df
    m = np.floor(my).astype(np.int64)

    def col(bb):
        return np.where(bb < nq, bb, np.where(bb == nb - 1, nq, -1))

    c0, c1 = col(m), col(m + 1)
    ok = (m >= 0) & (m + 1 <= nb - 1) & (m != seam) & (c0 >= 0) & (c1 >= 0)
    c0s, c1s = np.where(ok, c0, 0), np.where(ok, c1, 0)
    zn = bil(Z[S, c0s], Z[S, c1s], Z[S + 1, c0s], Z[S + 1, c1s], my - m, FX)
    take = ok & (zn >= zf)
    zc = np.where(take, Z[S, c0s], zc)
    q = (zc - cmin) / (cmax - cmin) * 256.0
    qf = np.where(q < 0.0, 0.0, np.where(q > 255.0, 255.0, np.floor(q)))
    out[:] = qf.astype(np.uint8)
    return out


def read_png_indexed(path: str):
    """Minimal PNG reader for the 8-bit palette PNGs libfmcw writes: (indices [H][W], palette [256][3])."""
    import struct
    import zlib
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, pal, W, H = 8, b"", None, 0, 0
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        crc = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0]
        assert zlib.crc32(typ + body) & 0xFFFFFFFF == crc, typ
        if typ == b"IHDR":
            W, H, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert depth == 8 and ctype == 3
        elif typ == b"PLTE":
            pal = np.frombuffer(body, np.uint8).reshape(-1, 3)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(H, W + 1)
    assert np.all(raw[:, 0] == 0)                   # filter type None on every row
    return raw[:, 1:].copy(), pal
