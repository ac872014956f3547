"""The reference's own scene files run unchanged (BASELINE.json configs[0]):
resources/data/cornell_box/scene.akari (importing cornell_box.akari, naming
CornellBox-Original.obj.mesh) and resources/example.akari (importing foo.akari) parse with the
restated .akari language (core/parser.cpp:150-363) into the scene the renderer's built-in
cornell_scene() restates — camera, Path node, material slots, geometry — pinned by the committed
golden resolution (tests/golden/reference_scenes.json, made by make_scene_golden.py from the files
themselves).  The live parse runs only where /root/reference is mounted."""
import json
import sys
from pathlib import Path

import numpy as np
import pytest

from akari_amd import scene
from conftest import CORNELL_MESH, GOLDEN

sys.path.insert(0, str(GOLDEN))
from scene_summary import summarize  # noqa: E402
import make_scene_golden  # noqa: E402

REF = Path("/root/reference/resources")
needs_ref = pytest.mark.skipif(not (REF / "data" / "cornell_box" / "scene.akari").exists(),
                               reason="reference tree not mounted")


def _golden():
    return json.loads((GOLDEN / "reference_scenes.json").read_text())


def test_golden_cornell_equals_builtin_cornell_scene():
    """The golden resolution of scene.akari is exactly cornell_scene() at the file's settings
    (1024^2, spp 16, max_depth 5, tile 1024) over the committed .mesh fixture."""
    g = _golden()["cornell_scene"]
    mine = summarize(scene.cornell_scene(CORNELL_MESH, resolution=(1024, 1024), spp=16, max_depth=5))
    mine = json.loads(json.dumps(mine))
    assert mine == g


def test_golden_cornell_compiles_to_the_reference_light_list():
    """SceneNode::compile (core/nodes/scene.cpp:51-92): the two emissive triangles of the light
    (material slot 7) become the area lights, with power 2 * area * uv-area * luminance(Le)."""
    cs = scene.compile_scene(scene.cornell_scene(CORNELL_MESH, resolution=(1024, 1024)))
    mi = np.asarray(_golden()["cornell_scene"]["shapes"][0]["material_indices"])
    assert sorted(np.asarray(cs.light_gid).tolist()) == np.flatnonzero(mi == 7).tolist()
    assert len(cs.power) == 2 and np.all(np.asarray(cs.power) > 0)


@needs_ref
def test_reference_scene_akari_parses_unchanged():
    sc = scene.load_scene_file(REF / "data" / "cornell_box" / "scene.akari")
    assert json.loads(json.dumps(summarize(sc))) == _golden()["cornell_scene"]
    # and renders the same scene as the built-in restatement: identical compiled arrays
    a = scene.compile_scene(sc)
    b = scene.compile_scene(scene.cornell_scene(CORNELL_MESH, resolution=(1024, 1024)))
    for f in ("vertices", "indices", "normals", "texcoords", "matid", "light_gid", "power"):
        assert np.array_equal(np.asarray(getattr(a, f)), np.asarray(getattr(b, f))), f
    assert a.camera == b.camera


@needs_ref
def test_reference_example_akari_parses_unchanged():
    """import ... as, $module.var references and a generic object node (example.akari:1-6)."""
    got = json.loads(json.dumps(make_scene_golden.example_summary(REF / "example.akari")))
    assert got == _golden()["example"]
    assert got["bar"] == [444.0, 123.0] and got["obj"]["fields"]["position"] == [1.0, 2.0, 3.0]
