"""Film output: Film::write_image semantics (core/film.h:97-113, GammaCorrection
common/color.h:58-61, 8-bit quantisation core/image.cpp:38-60), Python and C++ writers agreeing
byte for byte.  CPU only."""
import subprocess

import numpy as np

from akari_amd import capi, film
from conftest import ROOT


def _synthetic():
    w, h = 37, 23
    p = np.arange(w * h, dtype=np.int64)
    rad = np.stack([((p * 7 + c * 13) % 101).astype(np.float32) / np.float32(37.0) for c in range(3)], -1)
    rad[0, 0] = -1.0
    wt = np.where(p % 5 == 0, 0, p % 3 + 1).astype(np.float32)
    return rad.reshape(h, w, 3), wt.reshape(h, w)


def test_srgb_known_values():
    L = np.array([0.0, 0.002, 0.0031308, 0.18, 0.5, 1.0, 2.0, -0.5, np.nan], np.float32)
    s = film.linear_to_srgb(L)
    assert s[0] == 0 and s[1] == np.float32(0.002) * np.float32(12.92)
    assert abs(s[4] - 0.7353569) < 1e-6 and abs(s[5] - 1.0) < 1e-6
    q = film.quantize8(s)
    assert q.tolist()[:7] == [0, 7, 10, 118, 188, 255, 255] and q[7] == 0 and q[8] == 0
    # round(v * 255.5), half away from zero
    assert film.quantize8(np.array([0.51 / 255.5, 0.49 / 255.5, 254.6 / 255.5], np.float32)).tolist() == [1, 0, 255]


def test_resolve_divides_by_weight_only_when_nonzero():
    rad, wt = _synthetic()
    img = film.resolve(rad, wt)
    z = wt == 0
    assert np.array_equal(img[z], rad[z])
    assert np.array_equal(img[~z], (rad[~z] / wt[~z][:, None]).astype(np.float32))


def test_png_round_trip_and_cpp_writer_match(tmp_path):
    rad, wt = _synthetic()
    ref = film.to_srgb8(rad, wt)
    py_png = tmp_path / "py.png"
    film.write_png(py_png, rad, wt)
    assert np.array_equal(film.read_png_rgb8(py_png.read_bytes()), ref)
    exe = tmp_path / "film_png_demo"
    lib = capi.LIB_PATH.parent
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", str(ROOT / "tests" / "cpp" / "film_png_demo.cpp"),
                    "-o", str(exe), f"-L{lib}", "-lakr_hip", f"-Wl,-rpath,{lib}"], check=True)
    cpp_png, cpp_pfm = tmp_path / "cpp.png", tmp_path / "cpp.pfm"
    subprocess.run([str(exe), str(cpp_png), str(cpp_pfm)], check=True, timeout=60)
    assert np.array_equal(film.read_png_rgb8(cpp_png.read_bytes()), ref)
    py_pfm = tmp_path / "py.pfm"
    film.write_pfm(py_pfm, rad, wt)
    assert py_pfm.read_bytes() == cpp_pfm.read_bytes()
