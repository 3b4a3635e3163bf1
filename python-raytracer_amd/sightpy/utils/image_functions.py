"""Image asset loading (reference `utils/image_functions.py:7-33`).

Images are decoded with Pillow to uint8.  The float forms returned here keep the reference API;
the renderer itself uploads the *uint8* texels plus a 256-entry float64 table per texture
(`sightpy/_lower.py`), which reproduces `u8 / 256.0` (optionally linearised) bit for bit.
Relative asset paths are resolved against the working directory first (reference behaviour) and
then against this package's bundled `assets/` directory.
"""
from pathlib import Path

import numpy as np
from PIL import Image, ImageFilter

from .colour_functions import sRGB_to_sRGB_linear

__all__ = [
    "load_image",
    "load_image_with_blur",
    "load_image_as_linear_sRGB",
    "load_image_u8",
    "resolve_asset",
]

_ASSETS = Path(__file__).resolve().parent.parent / "assets"


def resolve_asset(path):
    """Map a reference-style path ('sightpy/textures/x.png') to an existing file."""
    p = Path(path)
    if p.exists():
        return p
    parts = p.parts
    if parts and parts[0] == "sightpy":
        parts = parts[1:]
    cand = _ASSETS.joinpath(*parts) if parts else _ASSETS
    if cand.exists():
        return cand
    raise FileNotFoundError("sightpy asset not found: %s (looked in CWD and %s)" % (path, _ASSETS))


def load_image_u8(path, blur=0.0):
    """Decode to a uint8 (H, W, C) array; the renderer's texel format."""
    img = Image.open(resolve_asset(path))
    if blur != 0.0:
        img = img.filter(ImageFilter.GaussianBlur(radius=blur))
    return np.asarray(img)


def load_image(path):
    return load_image_u8(path) / 256.0


def load_image_with_blur(path, blur=0.0):
    return load_image_u8(path, blur) / 256.0


def load_image_as_linear_sRGB(path, blur=0.0):
    print("proccesing " + Path(path).name)
    return sRGB_to_sRGB_linear(load_image_u8(path, blur) / 256.0)
