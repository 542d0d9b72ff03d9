"""GPU: spectrogram.png (radar_processing.m:331-348) rendered by
libfmcw (kernels_render.hip) and written as a palette PNG.

1. The rules: given the same float32 P, the GPU indices equal the numpy
   restatement (oracle/render.py) pixel for pixel (float64 arithmetic, same
   operation order, FMA contraction off in the kernel).
2. End to end: fmcw_stft_png on a slow-time signal against the restatement on
   the float64 oracle's P; fp32 rounding of P may move a colour-index boundary
   or a depth tie, so >= 99.5 % of the pixels agree and no pixel is off by more
   than one colour step except at depth ties (counted separately).
The pixels are parity-unpinned against MATLAB graphics (not runnable here)."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import render as R

pytestmark = pytest.mark.gpu


def _slow_signal(L, seed=0):
    rng = np.random.default_rng(seed)
    k = np.arange(L)
    x = np.abs(1.0 + 0.6 * np.sin(2 * np.pi * 37.0 * k / 1250.0) + 0.3 * np.sin(2 * np.pi * 90.0 * k / 1250.0)
               + 0.05 * rng.standard_normal(L))
    return x.astype(np.float32).astype(np.float64)


def _Q(P_nb_nseg, nq):
    """[nseg][nq + 1]: bins 0..nq-1 then the Nyquist bin."""
    P = np.asarray(P_nb_nseg).T
    return np.concatenate([P[:, :nq], P[:, -1:]], axis=1)


@pytest.mark.parametrize("L,nfft,W,H", [(1840, 2048, 640, 400), (900, 64, 300, 120), (3000, 0, 2906, 2038)])
def test_render_rules_exact(engine, L, nfft, W, H):
    import torch
    x = _slow_signal(L)
    prt = 8e-4
    fs = 1 / prt
    nfft = nfft or 2 ** O.nextpow2(L)
    win = O.stft_window("kaiser")
    _, Fv, T, P = O.spectrogram(x, win, 19, nfft, fs)
    P32 = P.astype(np.float32)
    nb = nfft // 2 + 1
    nq = nb - 1 if nfft == 64 else min(nb - 1, int(np.floor(150.0 / (fs / nfft))) + 2)
    Q = np.ascontiguousarray(_Q(P32, nq), np.float32)
    pmax = np.float32(P32.max())
    d_Q = torch.from_numpy(Q).cuda()
    d_nseg = torch.tensor([Q.shape[0]], dtype=torch.int64, device="cuda")
    d_pmax = torch.tensor([pmax], dtype=torch.float32, device="cuda")
    d_img = torch.empty((H, W + 1), dtype=torch.uint8, device="cuda")
    engine.render_spectrogram_device(d_Q, nq, d_nseg, d_pmax, nfft, fs, float(T[0]), float(T[1] - T[0]), W, H, d_img,
                                     stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    img = d_img.cpu().numpy()
    assert np.all(img[:, 0] == 0)
    want = R.render_indices(Q, nq, float(pmax), nfft, fs, float(T[0]), float(T[1] - T[0]), W, H)
    np.testing.assert_array_equal(img[:, 1:], want)
    assert len(np.unique(want)) > 20                  # a real picture, not one colour


def test_stft_png_end_to_end(engine, tmp_path):
    L, prt = 1840, 8e-4                               # 115 deployed frames x 16 chirps
    x = _slow_signal(L, seed=3)
    fs = 1 / prt
    path = tmp_path / "spectrogram.png"
    got = engine.stft_png(x, O.stft_window("kaiser"), 19, fs, str(path))
    idx, pal = R.read_png_indexed(str(path))
    assert idx.shape == (2038, 2906)                  # default: exportgraphics at 600 dpi of the default axes box
    assert got["png_bytes"] == path.stat().st_size
    np.testing.assert_array_equal(pal, R.jet_palette_u8())
    # the JSON-side outputs are those of fmcw_stft
    ref = O.spectrogram_pipeline(x, prt, O.stft_window("kaiser"), 19)
    sel = ref["intensity"].T > -80
    assert np.abs(got["intensity"][sel] - ref["intensity"].T[sel]).max() <= 1e-3
    # the picture against the restatement on the float64 oracle's P
    nfft = got["nfft"]
    _, Fv, T, P = O.spectrogram(x, O.stft_window("kaiser"), 19, nfft, fs)
    nq = min(nfft // 2, int(np.floor(150.0 / (fs / nfft))) + 2)
    want = R.render_indices(_Q(P, nq), nq, float(P.max()), nfft, fs, float(T[0]), float(T[1] - T[0]), 2906, 2038)
    same = np.mean(idx == want)
    assert same >= 0.995, same
    far = np.abs(idx.astype(int) - want.astype(int)) > 1
    assert np.mean(far) <= 0.002, np.mean(far)
