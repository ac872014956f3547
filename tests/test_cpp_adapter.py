"""The C++17 host adapter (akari_hip.hpp) builds against the C-ABI, and on the GPU renders the same
image as the Python binding of the same ABI."""
import subprocess

import numpy as np
import pytest

from akari_amd import capi, scene
from conftest import CORNELL_MESH, ROOT

SRC = ROOT / "tests" / "cpp" / "adapter_demo.cpp"


def _build(tmp_path):
    exe = tmp_path / "adapter_demo"
    lib = capi.LIB_PATH.parent
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", str(SRC), "-o", str(exe), f"-L{lib}", "-lakr_hip",
                    f"-Wl,-rpath,{lib}"], check=True)
    return exe


def test_adapter_compiles_and_links(tmp_path):
    assert _build(tmp_path).exists()


@pytest.mark.gpu
def test_adapter_render_matches_python_binding(tmp_path):
    exe = _build(tmp_path)
    out = tmp_path / "cornell.pfm"
    r = subprocess.run([str(exe), str(CORNELL_MESH), str(out), "32", "32", "4"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    assert "hit=1" in r.stdout and "geom=0" in r.stdout
    raw = out.read_bytes()
    header_end = raw.index(b"-1.0\n") + 5
    pfm = np.frombuffer(raw[header_end:], np.float32).reshape(32, 32, 3)[::-1]
    cs = scene.compile_scene(scene.cornell_scene(CORNELL_MESH, resolution=(32, 32)))
    with capi.HipContext(0) as ctx:
        scene.upload_scene(ctx, cs)
        rad, w = ctx.render(4, 5, [(0, 0, 32, 32)], 32, 32)
    assert np.array_equal(pfm, rad / w[..., None])


@pytest.mark.gpu
def test_adapter_ao_matches_python_binding(tmp_path):
    exe = _build(tmp_path)
    out = tmp_path / "cornell_ao.pfm"
    r = subprocess.run([str(exe), str(CORNELL_MESH), str(out), "32", "32", "4", "ao"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    raw = out.read_bytes()
    header_end = raw.index(b"-1.0\n") + 5
    pfm = np.frombuffer(raw[header_end:], np.float32).reshape(32, 32, 3)[::-1]
    cs = scene.compile_scene(scene.cornell_scene(CORNELL_MESH, resolution=(32, 32)))
    with capi.HipContext(0) as ctx:
        scene.upload_scene(ctx, cs)
        rad, w = ctx.render_ao(4, [(0, 0, 32, 32)], 32, 32)
    assert np.array_equal(pfm, rad / w[..., None])
