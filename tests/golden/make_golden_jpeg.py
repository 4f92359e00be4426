"""Generate tests/golden/jpeg_cases.npz: small JPEGs (Pillow / libjpeg-turbo encoder) and their libjpeg-turbo
decodes (Pillow), BGR.  Run: python tests/golden/make_golden_jpeg.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jpeg_cases import ENCODINGS, encode, image, reference_decode  # noqa: E402

out = {}
k = 0
for (H, W) in [(24, 40), (37, 53)]:
    for name, kw in ENCODINGS:
        data = encode(image(H, W, "smooth", seed=k), **kw)
        out[f"jpeg{k}"] = np.frombuffer(data, np.uint8)
        out[f"bgr{k}"] = reference_decode(data)
        k += 1
data = encode(image(24, 40, "smooth")[..., 1], quality=75)
out[f"jpeg{k}"] = np.frombuffer(data, np.uint8)
out[f"bgr{k}"] = reference_decode(data)
k += 1
out["n"] = np.array(k)
np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "jpeg_cases.npz"), **out)
print("wrote", k, "cases")
