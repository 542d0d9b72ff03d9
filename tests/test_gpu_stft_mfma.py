"""The STFT on the matrix cores against the VALU k_stft20 it replaces: P (:276, one-sided 'psd'),
max(P) (:282) and the direct 20 log10(P / max) (:283) bit for bit for k_stft_mfma (any nfft) and
k_stft64m (nfft 64, FMCW_STFT64_FOLD=0); the folded nfft-64 form k_stft64f (the default for
config 4: taps 10+k and 9-k paired, half the matrix work) to the fp32 dB bar.

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


def _run(engine, monkeypatch, mfma, x, hop, halo, store, nfft=NFFT, fold=False, win=None):
    import torch
    monkeypatch.setenv("FMCW_STFT_MFMA", "1" if mfma else "0")
    monkeypatch.setenv("FMCW_STFT64_FOLD", "1" if fold else "0")
    dev = "cuda"
    nfr = len(x) // PN
    slow = torch.from_numpy(x.reshape(nfr, PN)).to(dev)
    flist = torch.arange(nfr, dtype=torch.int32, device=dev)
    d_len = torch.tensor([len(x)], dtype=torch.int64, device=dev)
    win = torch.from_numpy((np.hanning(WLEN + 2)[1:-1] if win is None else win).astype(np.float32)).to(dev)
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
    n1, p1, m1 = _run(engine, monkeypatch, True, x, hop, hl, store, nfft)     # k_stft64m at nfft 64
    n0, p0, m0 = _run(engine, monkeypatch, False, x, hop, hl, store, nfft)
    assert n1 == n0 and n1 == (len(x) + (WLEN - 1 if halo else 0) - (WLEN - hop)) // hop
    np.testing.assert_array_equal(m1, m0)
    assert not np.isnan(p1).any()
    np.testing.assert_array_equal(p1, p0)        # P (stored pass) or the dB map (direct pass)


def _db(p, pm):
    with np.errstate(divide="ignore"):
        return 20 * np.log10(p.astype(np.float64) / np.float64(pm))   # :283 20 log10 of the power


def _truth_db(x, halo, w, hop):
    """fp64 P of every segment and bin (the 64-point DFT of the windowed 20-sample segment, one-sided
    'psd' scaling), as dB against its own maximum."""
    xx = np.concatenate([x, halo]) if halo is not None else x
    xx = xx.astype(np.float64)
    ns = (len(xx) - (WLEN - hop)) // hop
    X = np.lib.stride_tricks.sliding_window_view(xx, WLEN)[::hop][:ns]
    S = (X * w.astype(np.float32).astype(np.float64)) @ np.exp(-2j * np.pi * np.outer(np.arange(WLEN), np.arange(33)) / 64)
    P = np.abs(S) ** 2
    P[:, 1:32] *= 2
    return _db(P, P.max())


@pytest.mark.parametrize("frames,hop,halo,store,wkind", [(3, 1, False, True, "hann"), (7, 1, True, True, "hann"),
                                                          (5, 3, False, True, "kaiser"), (9, 1, False, False, "hann"),
                                                          (40, 1, False, False, "kaiser"), (2, 4, False, False, "rand"),
                                                          (4, 1, True, False, "rand")])
def test_folded_stft64_meets_the_db_bar(engine, monkeypatch, frames, hop, halo, store, wkind):
    """k_stft64f (default at nfft 64) against fp64: every output at or above -80 dB within 1e-3 dB
    (the fp32 STFT bar of tests/test_gpu_device_path.py), the bins below the floor finite and below
    it, max(P) within 2e-6 of k_stft20's (VALU).  The two fp32 forms differ from each other by up to
    twice the bar near the floor (each is within it of fp64), so they are not compared with each
    other.  Windows that are not bit-symmetric (kaiser(20, 3), a random one) included: the fold
    applies the taps to the samples, so it needs no symmetry."""
    from oracle import oracle as O
    rng = np.random.default_rng(frames * 7 + hop)
    x = (np.repeat(rng.uniform(0.5, 40.0, frames), PN) * (1 + 0.05 * rng.standard_normal(frames * PN))).astype(np.float32)
    x = np.abs(x)
    hl = (np.abs(rng.standard_normal(WLEN - 1)) * 20).astype(np.float32) if halo else None
    w = {"hann": O.stft_window("hann"), "kaiser": O.stft_window("kaiser"), "rand": rng.uniform(0.1, 1.0, WLEN)}[wkind]
    n1, p1, m1 = _run(engine, monkeypatch, True, x, hop, hl, store, 64, fold=True, win=w)
    n0, p0, m0 = _run(engine, monkeypatch, False, x, hop, hl, store, 64, win=w)
    assert n1 == n0 == (len(x) + (WLEN - 1 if halo else 0) - (WLEN - hop)) // hop
    assert abs(float(m1[0]) / float(m0[0]) - 1) <= 2e-6
    d1 = _db(p1, m1[0]) if store else p1.astype(np.float64)
    dt = _truth_db(x, hl, w, hop)
    assert dt.shape == d1.shape
    sel = dt >= -80
    assert sel.mean() > 0.2
    assert np.abs(d1[sel] - dt[sel]).max() <= 1e-3
    assert (d1[~sel] <= -80 + 1e-3).all() and not np.isnan(d1).any()


@pytest.mark.parametrize("L", [0, 1, 19, 20, 21, 83, 84, 85, 256])
def test_folded_stft64_short_signals(engine, monkeypatch, L):
    """k_stft64f at the edges of its 64-segment units and of the window: no segment (L < 20:
    nseg 0, max(P) stays 0, nothing written), one segment (L = 20), a unit's worth plus and minus
    one; both passes (max(P), then the direct dB map) against fp64 at the dB bar."""
    import torch
    from oracle import oracle as O
    monkeypatch.setenv("FMCW_STFT_MFMA", "1")
    monkeypatch.setenv("FMCW_STFT64_FOLD", "1")
    rng = np.random.default_rng(L + 5)
    x = np.abs(rng.standard_normal(PN) * 10 + 3).astype(np.float32)
    slow = torch.from_numpy(x.reshape(1, PN)).to("cuda")
    flist = torch.zeros(1, dtype=torch.int32, device="cuda")
    d_len = torch.tensor([L], dtype=torch.int64, device="cuda")
    w = O.stft_window("hann")
    win = torch.from_numpy(w.astype(np.float32)).to("cuda")
    max_seg = PN
    out = torch.full((max_seg, 33), np.nan, dtype=torch.float32, device="cuda")
    pmax = torch.zeros(1, dtype=torch.float32, device="cuda")
    nseg = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    engine.stft_power_device(slow, flist, d_len, PN, win, WLEN, WLEN - 1, 64, 1250.0, max_seg, None, pmax, nseg)
    engine.stft_db_direct_device(slow, flist, d_len, PN, win, WLEN, WLEN - 1, 64, 1250.0, max_seg, pmax, out)
    torch.cuda.synchronize()
    n = int(nseg.item())
    got = out.cpu().numpy()
    assert n == max(0, L - (WLEN - 1))
    assert np.isnan(got[n:]).all()                                          # nothing past nseg
    if n == 0:
        assert float(pmax.item()) == 0.0
        return
    dt = _truth_db(x[:L], None, w, 1)
    d1 = got[:n].astype(np.float64)
    sel = dt >= -80
    assert np.abs(d1[sel] - dt[sel]).max() <= 1e-3
    assert (d1[~sel] <= -80 + 1e-3).all()
