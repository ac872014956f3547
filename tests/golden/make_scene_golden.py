"""Golden resolution of the reference's own scene files, parsed unchanged by akari_amd.scene's
.akari parser (core/parser.cpp:150-363 restated): resources/data/cornell_box/scene.akari (+ the
cornell_box.akari it imports and the CornellBox-Original.obj.mesh it names) and
resources/example.akari (+ foo.akari).  The files stay in the reference tree; this writes only the
resolved values (JSON).  Run where /root/reference is mounted:
    python tests/golden/make_scene_golden.py"""
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))
sys.path.insert(0, str(HERE))

from akari_amd import scene as S  # noqa: E402
from scene_summary import summarize  # noqa: E402

REF = Path("/root/reference/resources")


def example_summary(path):
    mod = S.SdlParser().parse_file(path)
    obj = mod.exports["obj"]
    return {"bar": mod.exports["bar"], "obj": {"type": obj.type, "fields": obj.fields}}


def main():
    out = {
        "cornell_scene": summarize(S.load_scene_file(REF / "data" / "cornell_box" / "scene.akari")),
        "example": example_summary(REF / "example.akari"),
        "sources": ["resources/data/cornell_box/scene.akari", "resources/data/cornell_box/cornell_box.akari",
                    "resources/data/cornell_box/CornellBox-Original.obj.mesh", "resources/example.akari",
                    "resources/foo.akari"],
    }
    (HERE / "reference_scenes.json").write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print("wrote", HERE / "reference_scenes.json")


if __name__ == "__main__":
    main()
