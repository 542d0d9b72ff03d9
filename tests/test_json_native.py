"""CPU: the native jsonencode writer (libfmcw fmcw_json_write)
produces byte for byte what the Python mirror matlab_json.encode does, for the
shapes and values radar_processing.m writes (:302-436, :566-593)."""
import numpy as np
import pytest

from fmcw_radar_processing_amd import json_native
from fmcw_radar_processing_amd.matlab_json import encode


def _same(tmp_path, obj, pretty=True, threads=0):
    p = tmp_path / "x.json"
    n = json_native.write(p, obj, pretty=pretty, threads=threads)
    got = p.read_bytes()
    assert n == len(got)
    want = encode(obj, pretty=pretty).encode()
    assert got == want
    return got


@pytest.mark.parametrize("pretty", [True, False])
def test_shapes_and_values(tmp_path, pretty):
    rng = np.random.default_rng(3)
    obj = {
        "time": (np.arange(37) * 0.0008 + 0.008).astype(np.float32),     # 1xN float32 (GPU output)
        "frequency": np.logspace(0, 2.8, 11),                            # 1xN float64
        "intensity": (rng.standard_normal((5, 9)) * 30).astype(np.float32).T,   # strided (transposed) view
        "scalar": 100, "neg_zero": -0.0, "big": 1e15, "int_like": 123456789012.0,
        "tiny": 1.25e-7, "nan_inf": np.array([np.nan, np.inf, -np.inf, 2.5]),
        "column": np.arange(4.0).reshape(4, 1), "empty": np.zeros((0,)),
        "ints": np.arange(6), "one": np.array([[7.5]]),
        "title": 'All Frames - "Log-Scaled" \\ Spectrogram',
    }
    _same(tmp_path, obj, pretty)


@pytest.mark.parametrize("pretty", [True, False])
def test_logicals(tmp_path, pretty):
    """MATLAB logicals encode as true / false, scalars and arrays alike (jsonencode)."""
    obj = {"flag": True, "off": np.bool_(False), "mask": np.array([True, False, True]),
           "grid": np.array([[True, False], [False, False], [True, True]]), "col": np.array([[False], [True]])}
    got = _same(tmp_path, obj, pretty)
    import json
    d = json.loads(got)
    assert d["flag"] is True and d["off"] is False and d["mask"] == [True, False, True]
    assert d["grid"] == [[True, False], [False, False], [True, True]] and d["col"] == [False, True]


@pytest.mark.parametrize("threads", [1, 3, 0])
def test_large_arrays_cross_pieces(tmp_path, threads):
    """Vectors and matrices larger than one formatting piece (65536 elements)."""
    rng = np.random.default_rng(5)
    inten = (rng.standard_normal((70001, 3)) * 20 - 40).astype(np.float32)   # [nseg][nbins] -> 3 x 70001
    obj = {"time": np.arange(70001) * 0.0008, "intensity": inten.T,
           "rows": (rng.standard_normal((300, 400))).astype(np.float32), "filename": "f"}
    _same(tmp_path, obj, True, threads)


def test_spectrogram_file_layout(tmp_path):
    """spectrogram_data.json of :306-321 from the device layout [nseg][nbins]."""
    inten = np.linspace(-80, 0, 4 * 6, dtype=np.float32).reshape(4, 6)      # nseg 4, nbins 6
    obj = {"time": np.arange(4, dtype=np.float32), "frequency": np.arange(6, dtype=np.float32),
           "intensity": inten.T, "title": "All Frames - Log-Scaled Spectrogram",
           "xLabel": "Time (s)", "yLabel": "Frequency (Hz)"}
    got = _same(tmp_path, obj).decode()
    import json
    d = json.loads(got)
    assert list(d) == ["time", "frequency", "intensity", "title", "xLabel", "yLabel"]
    assert np.allclose(np.array(d["intensity"]), inten.T)


def test_bad_arguments(tmp_path):
    from fmcw_radar_processing_amd import FmcwError
    with pytest.raises(FmcwError, match="E_ARG"):
        json_native.write(tmp_path / "no" / "dir" / "x.json", {"a": 1})
    with pytest.raises(ValueError):
        json_native.write(tmp_path / "x.json", {"a": np.zeros((2, 2, 2))})
