"""Film output: the reference's Film::write_image (core/film.h:97-113) —
pixel = radiance / weight (radiance when weight is 0), GammaCorrection (linear_to_srgb,
common/color.h:58-61), clamp to [0, 1], 8-bit quantisation round(v * 255.5) (core/image.cpp:38-60)
— and a dependency-free PNG / PFM writer.  Host-side; the C++ adapter (akari_hip.hpp Film) does
the same, byte for byte.

pow is evaluated in f64 and rounded to f32: the correctly rounded powf the reference calls returns
the same value except in vanishingly rare halfway cases."""
from __future__ import annotations

import struct
import zlib
from pathlib import Path

import numpy as np


def resolve(radiance: np.ndarray, weight: np.ndarray) -> np.ndarray:
    """Film::write_image's pixel value: radiance / weight, or radiance where weight == 0."""
    radiance = np.asarray(radiance, np.float32)
    weight = np.asarray(weight, np.float32)[..., None]
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(weight != 0, radiance / np.where(weight != 0, weight, 1), radiance).astype(np.float32)


def linear_to_srgb(L: np.ndarray) -> np.ndarray:
    """select(L < 0.0031308, L * 12.92, 1.055 * pow(L, 1 / 2.4f) - 0.055) in f32."""
    L = np.asarray(L, np.float32)
    with np.errstate(invalid="ignore"):
        p = np.power(L.astype(np.float64), np.float64(np.float32(1.0) / np.float32(2.4))).astype(np.float32)
    hi = (np.float32(1.055) * p - np.float32(0.055)).astype(np.float32)
    return np.where(L < np.float32(0.0031308), (L * np.float32(12.92)).astype(np.float32), hi).astype(np.float32)


def quantize8(rgb: np.ndarray) -> np.ndarray:
    """clamp to [0, 1], then (uint8) clamp((int) round(v * 255.5), 0, 255)."""
    v = np.clip(np.nan_to_num(np.asarray(rgb, np.float32), nan=0.0), np.float32(0), np.float32(1))
    q = np.floor(v.astype(np.float64) * 255.5 + 0.5)  # round half away from zero (v >= 0)
    return np.clip(q, 0, 255).astype(np.uint8)


def to_srgb8(radiance: np.ndarray, weight: np.ndarray) -> np.ndarray:
    return quantize8(linear_to_srgb(resolve(radiance, weight)))


def png_bytes(rgb8: np.ndarray) -> bytes:
    """8-bit RGB PNG (filter 0 on every row)."""
    rgb8 = np.ascontiguousarray(rgb8, np.uint8)
    h, w, _ = rgb8.shape
    raw = b"".join(b"\x00" + rgb8[y].tobytes() for y in range(h))

    def chunk(tag: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) +
            chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))


def read_png_rgb8(data: bytes) -> np.ndarray:
    """Decoder for the 8-bit RGB, filter-0 PNGs written here and by the C++ adapter (tests)."""
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    w = h = 0
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        tag, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(tag + body) & 0xFFFFFFFF, "bad chunk CRC"
        if tag == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert depth == 8 and ctype == 2
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = np.frombuffer(raw, np.uint8).reshape(h, 1 + 3 * w)
    assert np.all(rows[:, 0] == 0), "only filter type 0 is produced"
    return rows[:, 1:].reshape(h, w, 3).copy()


def write_png(path, radiance: np.ndarray, weight: np.ndarray) -> None:
    Path(path).write_bytes(png_bytes(to_srgb8(radiance, weight)))


def write_pfm(path, radiance: np.ndarray, weight: np.ndarray) -> None:
    """Linear float map (bottom-up rows, little endian), pixel = radiance / weight."""
    img = resolve(radiance, weight)
    h, w, _ = img.shape
    Path(path).write_bytes(f"PF\n{w} {h}\n-1.0\n".encode() + np.ascontiguousarray(img[::-1], "<f4").tobytes())
