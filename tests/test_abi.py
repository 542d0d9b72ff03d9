"""CPU: the C-ABI library loads, exports every symbol include/fmcw.h declares,
validates arguments, and refuses to run without a gfx950 device (no fallback)."""
import ctypes as ct
import os
import re

import pytest

from fmcw_radar_processing_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fmcw.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|const char\*)\s+(fmcw_\w+)\s*\(", src, re.M)))


def test_header_declares_the_path():
    names = declared_functions()
    for must in ("fmcw_ctx_create", "fmcw_set_taps", "fmcw_process", "fmcw_range_fft", "fmcw_stft",
                 "fmcw_process_device", "fmcw_stft_power_device", "fmcw_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_functions()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding types every declared entry point, and nothing else
    assert sorted(_lib.SIGNATURES) == names


def test_abi_version_and_error_string():
    lib = _lib.load()
    assert lib.fmcw_abi_version() == _lib.ABI_VERSION == 4
    assert isinstance(lib.fmcw_last_error(), bytes)


def test_null_context_is_an_argument_error():
    lib = _lib.load()
    p = _lib.Params(64, 16, 256, 16, 1, 9, 211.2, 200, 50, 0.9, 25, 0.1875)
    assert lib.fmcw_process(None, ct.byref(p), None, 0, 1, *([None] * 8), 0, None) == _lib.FMCW_E_ARG
    assert lib.fmcw_ctx_destroy(None) == _lib.FMCW_OK


def test_ctx_create_validates_before_touching_a_device():
    lib = _lib.load()
    h = ct.c_void_p()
    assert lib.fmcw_ctx_create(0, None, ct.byref(h)) == _lib.FMCW_E_ARG       # no device at all
    assert lib.fmcw_ctx_create(65, None, ct.byref(h)) == _lib.FMCW_E_ARG
    assert lib.fmcw_ctx_create(1, None, None) == _lib.FMCW_E_ARG
    n = ct.c_int32()
    assert lib.fmcw_ctx_devices(None, ct.byref(n), None, None) == _lib.FMCW_E_ARG


def test_stft_size_rules_are_host_side():
    lib = _lib.load()
    ns, nf, nb = ct.c_int64(), ct.c_int32(), ct.c_int32()
    # :273 nfft = 2^nextpow2(L); ncol = fix((L - noverlap)/hop)
    assert lib.fmcw_stft_sizes(1840, 20, 19, 0, 1024, ct.byref(ns), ct.byref(nf), ct.byref(nb)) == 0
    assert (ns.value, nf.value, nb.value) == (1821, 2048, 1024)
    assert lib.fmcw_stft_sizes(2048, 20, 19, 0, 0, ct.byref(ns), ct.byref(nf), ct.byref(nb)) == 0
    assert (ns.value, nf.value, nb.value) == (2029, 2048, 1025)
    assert lib.fmcw_stft_sizes(500, 20, 19, 64, 0, ct.byref(ns), ct.byref(nf), ct.byref(nb)) == 0
    assert (ns.value, nf.value, nb.value) == (481, 64, 33)
    # MATLAB's spectrogram raises on a signal shorter than the window
    assert lib.fmcw_stft_sizes(10, 20, 19, 0, 1024, ct.byref(ns), ct.byref(nf), ct.byref(nb)) == _lib.FMCW_E_DATA
    assert b"shorter than the window" in lib.fmcw_last_error()
    assert lib.fmcw_stft_sizes(100, 20, 20, 0, 0, ct.byref(ns), ct.byref(nf), ct.byref(nb)) == _lib.FMCW_E_ARG


def test_no_cpu_fallback_without_a_device():
    """On a host without a gfx950 device the library fails loudly."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from fmcw_radar_processing_amd import FmcwError
    from fmcw_radar_processing_amd.engine import Engine
    with pytest.raises(FmcwError, match="E_HIP"):
        Engine(0)
    with pytest.raises(FmcwError, match="E_HIP"):
        Engine([0, 1])


@pytest.mark.parametrize("spec", ["0,x", "1,,2", "-1", "a"])
def test_default_devices_rejects_a_malformed_list(monkeypatch, spec):
    """FMCW_DEVICES (fmcw_default_devices, the MEX drop-in's device choice) is parsed before
    any device is asked about: a malformed list is an argument error on any host."""
    monkeypatch.setenv("FMCW_DEVICES", spec)
    lib = _lib.load()
    ids = (ct.c_int32 * 8)()
    n = ct.c_int32(-1)
    assert lib.fmcw_default_devices(8, ids, ct.byref(n)) == _lib.FMCW_E_ARG
    assert n.value == 0 and "FMCW_DEVICES" in lib.fmcw_last_error().decode()
    assert lib.fmcw_default_devices(0, ids, ct.byref(n)) == _lib.FMCW_E_ARG


def test_default_devices_without_a_device(monkeypatch):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    monkeypatch.delenv("FMCW_DEVICES", raising=False)
    lib = _lib.load()
    ids = (ct.c_int32 * 8)()
    n = ct.c_int32()
    assert lib.fmcw_default_devices(8, ids, ct.byref(n)) == _lib.FMCW_E_HIP


def test_missing_library_raises(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.FmcwError, match="not found"):
        _lib.load()


def test_stream_handles_of_device_calls():
    """engine._sided: None -> NULL (the context's own stream), a raw handle and a torch stream with
    a non-zero handle pass through unchanged; only torch's default stream (handle 0) is routed
    through a joined side stream (GPU-side: tests/test_gpu_fullsize.py)."""
    from fmcw_radar_processing_amd.engine import _sided

    class _S:                       # a torch.cuda.Stream stand-in with a non-default handle
        cuda_stream = 0x1234
    for arg, want in ((None, None), (7, 7), (_S(), 0x1234)):
        with _sided(arg) as h:
            assert h.value == want
