"""The nfft-64 STFT on the matrix cores (k_stft64m, kernels_stft.hip) against the VALU k_stft20
it replaces for config 4: P (:276, one-sided 'psd'), max(P) (:282) and the direct 20 log10(P / max) (:283) bit for bit.

An f32 MFMA is a k-ordered chain of f32 fmas, so each S(seg, bin) is the same chain over the
20 taps as k_stft20's loop; FMCW_STFT_MFMA=0 selects the VALU kernel.  nfft 64 runs the
33-bin layout (k_stft64m), any other nfft the 32-bin column chunks (k_stft_mfma).  Ragged segment counts
(partial 16-segment groups and 256-segment blocks), hop 1 and 3, a right halo (the multi-GPU
form), the P-storing pass, and the max-only pass followed by the direct dB pass.  Against the oracle the same path is held to
the dB bar by tests/test_gpu_device_path.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WLEN, NFFT, PN = 20, 64, 256


def _run(engine, monkeypatch, mfma, x, hop, halo, store, nfft=NFFT):
    import torch
    monkeypatch.setenv("FMCW_STFT_MFMA", "1" if mfma else "0")
    dev = "cuda"
    nfr = len(x) // PN
    slow = torch.from_numpy(x.reshape(nfr, PN)).to(dev)
    flist = torch.arange(nfr, dtype=torch.int32, device=dev)
    d_len = torch.tensor([len(x)], dtype=torch.int64, device=dev)
    win = torch.from_numpy(np.hanning(WLEN + 2)[1:-1].astype(np.float32)).to(dev)
    max_seg = len(x) + WLEN
    d_P = torch.full((max_seg, nfft // 2 + 1), np.nan, dtype=torch.float32, device=dev)
    pmax = torch.zeros(1, dtype=torch.float32, device=dev)
    nseg = torch.zeros(1, dtype=torch.int64, device=dev)
    d_halo = d_hl = None
    if halo is not None:
        d_halo = torch.from_numpy(halo).to(dev)
        d_hl = torch.tensor([len(halo)], dtype=torch.int64, device=dev)
    nh = 0 if halo is None else len(halo)
    engine.stft_power_device(slow, flist, d_len, PN, win, WLEN, WLEN - hop, nfft, 1250.0, max_seg,
                             d_P if store else None, pmax, nseg, d_halo=d_halo, n_halo=nh, d_halo_len=d_hl)
    if not store:   # the direct dB pass (bench.py --stft-form direct): P recomputed, 20 log10(P / max) written
        engine.stft_db_direct_device(slow, flist, d_len, PN, win, WLEN, WLEN - hop, nfft, 1250.0, max_seg, pmax,
                                     d_P, d_halo=d_halo, n_halo=nh, d_halo_len=d_hl)
    torch.cuda.synchronize()
    n = int(nseg.item())
    return n, d_P[:n].cpu().numpy(), pmax.cpu().numpy()


@pytest.mark.parametrize("frames,hop,halo,store,nfft", [(3, 1, False, True, 64), (7, 1, True, True, 64),
                                                         (5, 3, False, True, 64), (9, 1, False, False, 64),
                                                         (40, 1, False, True, 64), (3, 1, False, True, 256),
                                                         (5, 1, True, False, 2048), (4, 2, False, True, 512), (2, 1, False, True, 32)])
def test_mfma_stft_is_bit_identical(engine, monkeypatch, frames, hop, halo, store, nfft):
    rng = np.random.default_rng(frames * 10 + hop)
    # a slow-time magnitude signal: per-frame levels with noise, ragged length (a partial last frame)
    x = (np.repeat(rng.uniform(0.5, 40.0, frames), PN) * (1 + 0.05 * rng.standard_normal(frames * PN))).astype(np.float32)
    x = np.abs(x)
    hl = (np.abs(rng.standard_normal(WLEN - 1)) * 20).astype(np.float32) if halo else None
    n1, p1, m1 = _run(engine, monkeypatch, True, x, hop, hl, store, nfft)
    n0, p0, m0 = _run(engine, monkeypatch, False, x, hop, hl, store, nfft)
    assert n1 == n0 and n1 == (len(x) + (WLEN - 1 if halo else 0) - (WLEN - hop)) // hop
    np.testing.assert_array_equal(m1, m0)
    assert not np.isnan(p1).any()
    np.testing.assert_array_equal(p1, p0)        # P (stored pass) or the dB map (direct pass)
