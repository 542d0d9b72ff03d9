"""CPU: the host-threaded writers under AddressSanitizer + UBSan and ThreadSanitizer
(SURVEY 5 "Race detection / sanitizers").

json_writer.cpp (16 formatter threads) and png_writer.cpp (parallel deflate strips) are
built with the host compiler by csrc/Makefile targets `asan` and `tsan`, linked with the
driver tests/native/sanitize_writers.cpp, and run at several thread counts.  Any sanitizer
report fails the test (halt_on_error, non-zero exit).  The files they write are then checked
byte for byte against the Python mirror (matlab_json.encode: jsonencode of :306-321 /
:355-361 shapes) and the PNG rows decoded back (oracle/render.py's reader), so the
sanitized code is the code that writes the right bytes.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from fmcw_radar_processing_amd.matlab_json import encode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fmcw_radar_processing_amd", "csrc")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None,
                                reason="needs the host C++ toolchain")


@pytest.fixture(scope="module")
def binaries():
    r = subprocess.run(["make", "-s", "-C", CSRC, "asan", "tsan"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return {k: os.path.join(CSRC, "build", f"san_{k}") for k in ("asan", "tsan")}


def _expected():
    nseg, nb = 3001, 1024
    s = np.arange(nseg)[:, None]
    b = np.arange(nb)[None, :]
    v = (s * 7 + b * 13) % 1000
    inten = np.where(v == 999, np.nan, np.where(v == 998, np.inf, v / 8.0 - 60.0)).astype(np.float32)
    spec = {"time": (np.arange(nseg, dtype=np.float32) + 10) / np.float32(1250.0),
            "frequency": (np.arange(nb) + 1) * 0.125,
            "intensity": inten.T,                                   # [nseg][nbins] -> nbins x nseg
            "title": "All Frames - Log-Scaled Spectrogram"}
    F, nr = 115, 256
    i = np.arange(F)[:, None]
    r = np.arange(nr)[None, :]
    prof = (((i * 31 + r * 17) % 4096) / 16.0).astype(np.float32)
    rf = {"range_tx1rx1_max_abs": prof.T, "target_bin": ((np.arange(F) * 37) % nr).astype(np.int32),
          "detected": (np.arange(F) % 3) != 0, "filename": "radar_data"}
    W, H = 2906, 2038
    x = np.arange(W)[None, :]
    y = np.arange(H)[:, None]
    img = ((x // 7 + y // 5 + (x * y) % 3) & 255).astype(np.uint8)
    return spec, rf, img


@pytest.mark.parametrize("kind", ["asan", "tsan"])
@pytest.mark.parametrize("threads", [16, 3])
def test_writers_clean_under_sanitizer(binaries, tmp_path, kind, threads):
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    r = subprocess.run([binaries[kind], str(tmp_path), str(threads)], capture_output=True, text=True, env=env,
                       timeout=600)
    report = r.stderr
    assert r.returncode == 0 and "Sanitizer" not in report and "runtime error" not in report, report[-4000:]
    spec, rf, img = _expected()
    assert (tmp_path / "spectrogram_data.json").read_bytes() == encode(spec, pretty=True).encode()
    assert (tmp_path / "range_fft_data.json").read_bytes() == encode(rf, pretty=False).encode()
    from oracle import render as RR
    got, pal = RR.read_png_indexed(str(tmp_path / "spectrogram.png"))
    np.testing.assert_array_equal(got, img)
