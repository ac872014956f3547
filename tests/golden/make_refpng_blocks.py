"""Golden data from the reference's own output image resources/data/cornell_box/ref.png (512^2
sRGB8, render settings unknown): per 16x16-pixel block the mean per channel and the mean and
within-block variance of the grey level (channel mean), plus the global mean per channel, for the
statistical pin of the oracle and the HIP render (tests/test_oracle_kat.py, tests/test_gpu_parity.py;
the image itself stays in the reference tree).  Run where /root/reference is mounted:
    python tests/golden/make_refpng_blocks.py"""
import json
from pathlib import Path

import numpy as np
from PIL import Image

SRC = Path("/root/reference/resources/data/cornell_box/ref.png")
OUT = Path(__file__).resolve().parent / "ref_png_blocks.json"

ref = np.asarray(Image.open(SRC).convert("RGB")).astype(np.float64)
assert ref.shape == (512, 512, 3)
blocks = ref.reshape(32, 16, 32, 16, 3).mean(axis=(1, 3))
grey = ref.mean(axis=2).reshape(32, 16, 32, 16)
OUT.write_text(json.dumps({"source": "resources/data/cornell_box/ref.png", "block": 16,
                           "mean": ref.mean(axis=(0, 1)).round(4).tolist(),
                           "blocks": blocks.round(3).tolist(),
                           "grey_mean": grey.mean(axis=(1, 3)).round(4).tolist(),
                           "grey_var": grey.var(axis=(1, 3), ddof=1).round(4).tolist()}))
print(f"wrote {OUT}")
