"""GPU: fmcw_process_slow_device (ABI 4) -- the per-frame stages plus the start of the slow-time
leg in one call: the compaction of radar_processing.m:257-260 (k_compact's frame list and L) and
the reset of the STFT's running max(P) (:276, :282), run inside the detection kernel's last
workgroup on the single-pass schedule (as launches of their own on the streams schedule).

Its outputs must be the bits of fmcw_process_device followed by fmcw_compact_device: one chunk,
several chunks (the last chunk's kernel compacts every frame of the call), more than 4096 frames
(the scan's passes), the streams schedule, and the forced in-wave slow-time fix (the rare row that
was not a group candidate, now recomputed by the frame's own wave instead of a k_slow_fix launch).
"""
import numpy as np
import pytest

from fmcw_radar_processing_amd import FMCW_C32H, FMCW_C64, FMCW_PIPE_AUTO, FMCW_PIPE_STREAMS
from fmcw_radar_processing_amd import params as P
from oracle import oracle as O
from tests.helpers import TOL_FP32_REL_L2, case, rel_l2

pytestmark = pytest.mark.gpu


def _outs(torch, F, cfg, dev):
    M = cfg.max_targets
    return dict(profile=torch.full((F, cfg.nr), np.nan, device=dev),
                tgt_count=torch.full((F,), -3, dtype=torch.int32, device=dev),
                tgt_range_idx=torch.full((F, M), -3, dtype=torch.int32, device=dev),
                tgt_range_mag=torch.full((F, M), np.nan, device=dev),
                tgt_doppler_idx=torch.full((F, M), -3, dtype=torch.int32, device=dev),
                slow_mag=torch.full((F, cfg.pn), np.nan, device=dev))


def _both(engine, cfg, d_iq, F, dt=FMCW_C64):
    """(reference: process_device + compact_device, fused: process_slow_device) on the same input."""
    import torch
    dev, s = "cuda", torch.cuda.current_stream()
    res = []
    for fused in (False, True):
        outs = _outs(torch, F, cfg, dev)
        d_rd = torch.full((F, cfg.nr, cfg.nd, 2), np.nan, dtype=torch.float16 if dt == FMCW_C32H else torch.float32,
                          device=dev)
        flist = torch.full((F,), -7, dtype=torch.int32, device=dev)
        d_len = torch.full((1,), -1, dtype=torch.int64, device=dev)
        pmax = torch.full((1,), 123.0, dtype=torch.float32, device=dev)
        if fused:
            engine.process_slow_device(d_iq, F, dt, outs, flist, d_len, d_pmax=pmax, d_rd=d_rd, out_dtype=dt, stream=s)
        else:
            engine.process_device(d_iq, F, dt, outs, d_rd=d_rd, out_dtype=dt, stream=s)
            engine.compact_device(outs["tgt_count"], F, flist, d_len, stream=s)
        torch.cuda.synchronize()
        engine.synchronize()
        got = {k: v.cpu().numpy() for k, v in outs.items()}
        n = int((got["tgt_count"] > 0).sum())
        got.update(rd=d_rd.cpu().numpy(), frame_list=flist.cpu().numpy()[:n], L=int(d_len.item()),
                   pmax=float(pmax.item()))
        res.append(got)
    return res


def _check_same(ref, got, cfg):
    for k in ("profile", "tgt_count", "tgt_range_idx", "tgt_range_mag", "tgt_doppler_idx", "slow_mag", "rd",
              "frame_list"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    assert got["L"] == ref["L"] == cfg.pn * int((ref["tgt_count"] > 0).sum())
    assert got["pmax"] == 0.0 and ref["pmax"] == 123.0


def _frame0_with_gaps(cfg, F, frame0, need_empty=2):
    """The first frame0' >= frame0 whose F frames hold at least need_empty without a target."""
    dpb = cfg.dist_per_bin
    while sum(O.synth_frame_params(frame0 + i, cfg.nr, cfg.nd, dpb)["A"] == 0 for i in range(F)) < need_empty:
        frame0 += 1
    return frame0


def _synth(engine, cfg, F, dt=FMCW_C64, frame0=0):
    import torch
    if F < 1000:
        frame0 = _frame0_with_gaps(cfg, F, frame0)
    d_iq = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=torch.float16 if dt == FMCW_C32H else torch.float32,
                       device="cuda")
    engine.synth_device(d_iq, frame0, F, dt, stream=torch.cuda.current_stream())
    return d_iq


@pytest.mark.parametrize("F,chunk,pipe", [(24, 0, FMCW_PIPE_AUTO), (61, 9, FMCW_PIPE_AUTO), (40, 0, FMCW_PIPE_STREAMS),
                                          (5000, 0, FMCW_PIPE_AUTO), (5000, 2048, FMCW_PIPE_AUTO)])
def test_slow_leg_is_process_then_compact(engine, F, chunk, pipe):
    cfg = P.config(3)
    engine.set_taps(cfg, P.synth_calibration(cfg.nts))
    engine.set_pipeline(pipe)
    engine.set_chunk_frames(chunk)
    try:
        d_iq = _synth(engine, cfg, F, frame0=77)
        ref, got = _both(engine, cfg, d_iq, F)
    finally:
        engine.set_chunk_frames(0)
        engine.set_pipeline(FMCW_PIPE_AUTO)
    assert 0 < len(ref["frame_list"]) < F                  # frames with and without a target
    _check_same(ref, got, cfg)


def test_slow_leg_fp16_storage(engine):
    cfg = P.config(3)
    engine.set_taps(cfg, P.synth_calibration(cfg.nts))
    d_iq = _synth(engine, cfg, 48, FMCW_C32H, frame0=5)
    ref, got = _both(engine, cfg, d_iq, 48, FMCW_C32H)
    _check_same(ref, got, cfg)


def test_slow_leg_forced_fix_in_wave(engine, monkeypatch):
    """Every slow-time row through the in-wave direct DFT (FMCW_ONEPASS_FORCE_FIX=1 keeps no group
    candidates): the rows meet the fp32 bar against the oracle, the rest is unchanged."""
    import torch
    cfg, p, wr, wd, cal = case(1024, 256, 1024, 256, P.THROUGHPUT)
    F = 11
    iq = O.synth_frames(F, 256, 1024, 1024, 256, p["dist_per_bin"], frame0=321)
    engine.set_taps(cfg, cal, wr, wd)
    d_iq = torch.from_numpy(np.ascontiguousarray(iq).view(np.float32).reshape(F, 256, 1024, 2)).to("cuda")
    _, plain = _both(engine, cfg, d_iq, F)
    monkeypatch.setenv("FMCW_ONEPASS_FORCE_FIX", "1")
    _, fixed = _both(engine, cfg, d_iq, F)
    ref = O.process_frames(iq, cal, p, wr, wd)
    for k in ("tgt_count", "tgt_range_idx", "tgt_doppler_idx", "frame_list"):
        np.testing.assert_array_equal(fixed[k], plain[k], err_msg=k)
    np.testing.assert_array_equal(fixed["tgt_count"], ref["tgt_count"])
    det = ref["tgt_count"] > 0
    assert det.sum() >= 5
    err = rel_l2(fixed["slow_mag"][det], ref["slow_mag"][det], axis=1)
    assert err.max() <= TOL_FP32_REL_L2, err


@pytest.mark.parametrize("fold", ["1", "0"], ids=["k_stft64f", "k_stft64m"])
@pytest.mark.parametrize("direct", [False, True], ids=["stored_P", "direct_dB"])
def test_stft64_cached_table_follows_the_window(engine, direct, fold, monkeypatch):
    """The nfft-64 device calls keep their W table while the window pointer is unchanged; a window
    rewritten in place (same pointer) must still be used: k_stft64m (FMCW_STFT64_FOLD=0) checks the
    taps stored behind the table and forms its W entries itself when they differ; k_stft64f (the
    default) applies the taps to the samples and never reads the table."""
    import torch
    monkeypatch.setenv("FMCW_STFT64_FOLD", fold)
    dev, s = "cuda", torch.cuda.current_stream()
    rng = np.random.default_rng(4)
    pn, nfr = 256, 9
    slow = torch.from_numpy((np.abs(rng.standard_normal((nfr, pn))) * 30).astype(np.float32)).to(dev)
    flist = torch.arange(nfr, dtype=torch.int32, device=dev)
    d_len = torch.tensor([nfr * pn], dtype=torch.int64, device=dev)
    max_seg = nfr * pn - 19
    fs = 1250.0
    win = torch.tensor(O.stft_window("hann"), dtype=torch.float32, device=dev)

    def run():
        pmax = torch.zeros(1, dtype=torch.float32, device=dev)
        nseg = torch.zeros(1, dtype=torch.int64, device=dev)
        out = torch.full((max_seg, 33), np.nan, dtype=torch.float32, device=dev)
        if direct:
            engine.stft_power_device(slow, flist, d_len, pn, win, 20, 19, 64, fs, max_seg, None, pmax, nseg, stream=s)
            engine.stft_db_direct_device(slow, flist, d_len, pn, win, 20, 19, 64, fs, max_seg, pmax, out, stream=s)
        else:
            engine.stft_power_device(slow, flist, d_len, pn, win, 20, 19, 64, fs, max_seg, out, pmax, nseg, stream=s)
            engine.stft_db_device(out, nseg, max_seg, 64, fs, pmax, 0, out, stream=s)
        torch.cuda.synchronize()
        return out.cpu().numpy(), float(pmax.item())

    a1, m1 = run()
    a2, m2 = run()                                   # the cached table: same bits
    np.testing.assert_array_equal(a2, a1)
    assert m1 == m2
    win.copy_(torch.tensor(O.stft_window("kaiser"), dtype=torch.float32, device=dev))   # same pointer
    b1, mb = run()
    x = slow.cpu().numpy().reshape(-1).astype(np.float64)
    ref = O.spectrogram_pipeline(x, 1.0 / fs, O.stft_window("kaiser"), 19, nfft=64, nbins=0)["intensity"].T
    sel = ref > -80
    assert np.abs(b1[sel] - ref[sel]).max() <= 1e-3
    win2 = torch.tensor(O.stft_window("kaiser"), dtype=torch.float32, device=dev)   # a fresh pointer: a fresh table
    win, win_old = win2, win
    b2, mb2 = run()
    np.testing.assert_array_equal(b2, b1)
    assert mb == mb2



@pytest.mark.parametrize("fold", ["1", "0"], ids=["k_stft64f", "k_stft64m"])
def test_stft64_table_after_another_nfft_on_the_stream(engine, fold, monkeypatch):
    """One window pointer, one stream: an nfft-128 call rewrites the stream's table entry, so the
    next nfft-64 call must not take the entry as its cached nfft-64 table (the key is
    cleared by every writer).  The nfft-64 result after the detour equals the one before it."""
    import torch
    monkeypatch.setenv("FMCW_STFT64_FOLD", fold)
    dev, s = "cuda", torch.cuda.current_stream()
    rng = np.random.default_rng(7)
    pn, nfr = 256, 5
    slow = torch.from_numpy((np.abs(rng.standard_normal((nfr, pn))) * 30).astype(np.float32)).to(dev)
    flist = torch.arange(nfr, dtype=torch.int32, device=dev)
    d_len = torch.tensor([nfr * pn], dtype=torch.int64, device=dev)
    max_seg = nfr * pn - 19
    win = torch.tensor(O.stft_window("kaiser"), dtype=torch.float32, device=dev)

    def run(nfft):
        nb = nfft // 2 + 1
        pmax = torch.zeros(1, dtype=torch.float32, device=dev)
        nseg = torch.zeros(1, dtype=torch.int64, device=dev)
        out = torch.full((max_seg, nb), np.nan, dtype=torch.float32, device=dev)
        engine.stft_power_device(slow, flist, d_len, pn, win, 20, 19, nfft, 1250.0, max_seg, out, pmax, nseg, stream=s)
        torch.cuda.synchronize()
        return out.cpu().numpy(), float(pmax.item())

    a, ma = run(64)
    run(128)
    b, mb = run(64)
    np.testing.assert_array_equal(b, a)
    assert ma == mb
    x = slow.cpu().numpy().reshape(-1).astype(np.float64)
    P = O.spectrogram(x, O.stft_window("kaiser"), 19, 64, 1250.0)[3].T       # [seg][33], float64
    np.testing.assert_allclose(b, P, rtol=1e-4, atol=1e-6 * float(P.max()))


@pytest.mark.parametrize("direct", [False, True], ids=["stored_P", "direct_dB"])
def test_stft64_unaligned_output(engine, direct):
    """An output that is not 16-byte aligned (a caller's slice, fmcw.h sets no alignment rule for
    d_P / d_out) takes the table form instead of the 16-byte stores of k_stft64f / k_stft64m (ADVICE
    r05): same dB as the aligned call within the fp32 bar, nothing written outside the slice."""
    import torch
    dev, s = "cuda", torch.cuda.current_stream()
    rng = np.random.default_rng(11)
    pn, nfr = 256, 6
    slow = torch.from_numpy((np.abs(rng.standard_normal((nfr, pn))) * 30).astype(np.float32)).to(dev)
    flist = torch.arange(nfr, dtype=torch.int32, device=dev)
    d_len = torch.tensor([nfr * pn], dtype=torch.int64, device=dev)
    max_seg = nfr * pn - 19
    fs = 1250.0
    win = torch.tensor(O.stft_window("hann"), dtype=torch.float32, device=dev)

    def run(off):
        pmax = torch.zeros(1, dtype=torch.float32, device=dev)
        nseg = torch.zeros(1, dtype=torch.int64, device=dev)
        buf = torch.full((max_seg * 33 + 8,), -7.0, dtype=torch.float32, device=dev)
        out = buf[off:off + max_seg * 33].view(max_seg, 33)
        assert (out.data_ptr() % 16 == 0) == (off % 4 == 0)
        if direct:
            engine.stft_power_device(slow, flist, d_len, pn, win, 20, 19, 64, fs, max_seg, None, pmax, nseg, stream=s)
            engine.stft_db_direct_device(slow, flist, d_len, pn, win, 20, 19, 64, fs, max_seg, pmax, out, stream=s)
        else:
            engine.stft_power_device(slow, flist, d_len, pn, win, 20, 19, 64, fs, max_seg, out, pmax, nseg, stream=s)
            engine.stft_db_device(out, nseg, max_seg, 64, fs, pmax, 0, out, stream=s)
        torch.cuda.synchronize()
        b = buf.cpu().numpy()
        return b[off:off + max_seg * 33].reshape(max_seg, 33), np.concatenate([b[:off], b[off + max_seg * 33:]])

    a0, _ = run(0)
    a1, rest = run(1)
    assert np.all(rest == -7.0)
    x = slow.cpu().numpy().reshape(-1).astype(np.float64)
    ref = O.spectrogram_pipeline(x, 1.0 / fs, O.stft_window("hann"), 19, nfft=64, nbins=0)["intensity"].T
    sel = ref > -80
    for a in (a0, a1):
        assert np.isfinite(a).all()
        assert np.abs(a[sel] - ref[sel]).max() <= 1e-3


def test_host_stft_nfft64_peaks_at_0_dB(engine):
    """The host call at nfft 64 with the log-frequency output: its max(P) pass and its listed-bins
    pass form P the same way, so no intensity exceeds 0 dB (MATLAB: P / max(P) <= 1 exactly) beyond
    the one rounding of P * (1 / max(P)) (< 1e-6 dB), and the peak is near 0 dB."""
    rng = np.random.default_rng(5)
    x = (np.abs(rng.standard_normal(40)) * 10).astype(np.float32)  # 2^nextpow2(40) = 64
    w = O.stft_window("kaiser").astype(np.float32)
    out = engine.stft(x, w, 19, 1250.0, nfft=0, n_log_bins=1024)
    assert out["nfft"] == 64
    assert -3.0 < np.nanmax(out["intensity"]) <= 1e-6
