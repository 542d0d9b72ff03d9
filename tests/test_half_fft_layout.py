"""Index algebra of k_rdx's half-frame A/B build (-DXK_HALF, kernels_xcd.hip, profiles/r06_half_ab.txt).

Each wave of a pair runs a 512-point FFT of its parity's samples (n = 2 m + e, m = lane + 64 i) as DFT8
over i -> twiddle W512^(lane k1) -> LDS transpose (row stride 72) -> DFT8 over l1 -> twiddle
W64^(l0 s1) -> LDS transpose (element s1 97 + 8 k1 + 4 (k1 >> 2) + l0) -> DFT8 over l0, and the pair
combines X[r'] = E[r'] + W1024^r' O[r'], X[r' + 512] = E[r'] - W1024^r' O[r'], group g of the half
slot holding bins 32 g .. 32 g + 31.  This replays those exact index formulas and twiddle exponents
(fmcw_api.cpp build_xcd_tab's XT_H1 / XT_H2 / XT_HC) in numpy and checks (a) the result is the
1024-point FFT in the slot order xcd_bin(g, p) = 32 g + p of the half build, (b) both transposes
are bank-conflict-free under MI355X_MICROARCH.md's table (ds_write_b64: 4 x 16 lanes, banks
(a/4) mod 32; ds_read_b64: 2 x 32 lanes, (a/4) mod 64).  Host logic only: the kernel itself is
checked against the oracle on the GPU by the A/B call that times it.
"""
import numpy as np

from tests.test_lds_banks import extra_cycles

N = 1024


def w1024(e):
    return np.exp(-2j * np.pi * (e % N) / N)


def half_fft(x):
    """The half build's data flow for one chirp; returns the slot image [32 groups][32 positions]."""
    out = np.zeros((32, 32), complex)
    F = {}
    for e in (0, 1):
        z = np.array([[x[2 * (l + 64 * i) + e] for i in range(8)] for l in range(64)])
        z = np.fft.fft(z, axis=1)                                   # DFT8 over i -> k1
        for l in range(64):
            for k1 in range(1, 8):
                z[l, k1] *= w1024(2 * l * k1)                        # XT_H1: W512^(l k1)
        rt = np.zeros(1216, complex)
        for l in range(64):
            for k1 in range(8):
                rt[k1 * 72 + l] = z[l, k1]                           # T1 write
        u = np.array([[rt[(L >> 3) * 72 + (L & 7) + 8 * l1] for l1 in range(8)] for L in range(64)])
        u = np.fft.fft(u, axis=1)                                   # DFT8 over l1 -> s1
        for L in range(64):
            for s1 in range(1, 8):
                u[L, s1] *= w1024(16 * ((L & 7) * s1))               # XT_H2: W64^(l0 s1)
        rt = np.zeros(1216, complex)
        for L in range(64):
            for s1 in range(8):
                rt[s1 * 97 + L + 4 * (L >> 5)] = u[L, s1]            # T2 write
        v = np.array([[rt[(L >> 3) * 97 + 8 * (L & 7) + 4 * ((L & 7) >> 2) + l0] for l0 in range(8)]
                      for L in range(64)])
        F[e] = np.fft.fft(v, axis=1)                                # DFT8 over l0 -> s2
    for e in (0, 1):
        for L in range(64):
            for s2 in range(8):
                t = w1024(L + 64 * s2) * F[1][L, s2]                 # XT_HC: W1024^(lane + 64 s2)
                val = F[0][L, s2] + t if e == 0 else F[0][L, s2] - t
                out[16 * e + 2 * s2 + (L >> 5), L & 31] = val
    return out


def test_half_build_computes_the_fft_in_slot_order():
    rng = np.random.default_rng(7)
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    got = half_fft(x).reshape(-1)                                   # group-major = bin order 32 g + p
    want = np.fft.fft(x)
    assert np.abs(got - want).max() <= 1e-9 * np.abs(want).max()


def test_half_build_transposes_are_conflict_free():
    lanes = range(64)
    for k1 in range(8):                                             # T1 write (ds_write_b64)
        assert extra_cycles([k1 * 72 + l for l in lanes], 16, 32) == 0
    for l1 in range(8):                                             # T1 read (ds_read_b64)
        assert extra_cycles([(L >> 3) * 72 + (L & 7) + 8 * l1 for L in lanes], 32, 64) == 0
    for s1 in range(8):                                             # T2 write
        assert extra_cycles([s1 * 97 + L + 4 * (L >> 5) for L in lanes], 16, 32) == 0
    for l0 in range(8):                                             # T2 read
        assert extra_cycles([(L >> 3) * 97 + 8 * (L & 7) + 4 * ((L & 7) >> 2) + l0 for L in lanes], 32, 64) == 0
    for s2 in range(8):                                             # the pair's exchange, both ways
        assert extra_cycles([s2 * 64 + L for L in lanes], 16, 32) == 0
        assert extra_cycles([s2 * 64 + L for L in lanes], 32, 64) == 0


def test_a_naive_t2_layout_would_conflict():
    # the 4 (k1 >> 2) term is what makes T2's read conflict-free: without it k1 and k1 + 4 share banks
    lanes = range(64)
    assert sum(extra_cycles([(L >> 3) * 97 + 8 * (L & 7) + l0 for L in lanes], 32, 64) for l0 in range(8)) > 0
