"""Seam-aware blur of a 4x3 cube-cross skybox (reference `backgrounds/util/blur_background.py:17-132`).

Each face is blurred on a 3N x 3N canvas holding the face in the centre and its four neighbours
(rotated so their shared edges line up), with Pillow's GaussianBlur, then cropped back.  The
reference builds the canvases from `u8/256` floats and converts them to images with
`(255 * x).astype(uint8)`; that conversion only depends on the byte, so it is applied to the
texels up front here.  The result is returned as uint8 (the device texel format); the reference
returns `sRGB_to_sRGB_linear(blurred / 256)`, which is exactly the device's `lut[byte]`.
"""
import numpy as np
from PIL import Image, ImageFilter

from ...utils.colour_functions import sRGB_to_sRGB_linear

__all__ = ["blur_skybox", "blur_skybox_u8"]

# canvas slots: (row block, col block) of a 3x3 grid of N x N tiles
_W, _C, _E, _S, _NTH = (1, 0), (1, 1), (1, 2), (2, 1), (0, 1)

# for each face: {slot: (face, quarter turns passed to np.rot90)}; faces named by cross position
_LAYOUTS = {
    "front": {_W: ("left", 0), _C: ("front", 0), _E: ("right", 0), _S: ("bottom", 0), _NTH: ("top", 0)},
    "right": {_W: ("front", 0), _C: ("right", 0), _E: ("back", 0), _S: ("bottom", 1), _NTH: ("top", -1)},
    "back": {_W: ("right", 0), _C: ("back", 0), _E: ("left", 0), _S: ("bottom", 2), _NTH: ("top", 2)},
    "left": {_W: ("back", 0), _C: ("left", 0), _E: ("front", 0), _S: ("bottom", -1), _NTH: ("top", 1)},
    "top": {_W: ("left", -1), _C: ("top", 0), _E: ("right", 1), _S: ("front", 0), _NTH: ("back", 2)},
    "bottom": {_W: ("left", 1), _C: ("bottom", 0), _E: ("right", -1), _S: ("back", 2), _NTH: ("front", 0)},
}
# where each face sits in the 4x3 cross (row block, col block)
_CROSS = {"left": (1, 0), "front": (1, 1), "right": (1, 2), "back": (1, 3), "top": (0, 1), "bottom": (2, 1)}


def blur_skybox_u8(cross_u8, blur, cubemap=""):
    """uint8 (3N, 4N, 3) cube cross -> uint8 (3N, 4N, 3) blurred cross."""
    print("blurring " + cubemap)
    n = int(cross_u8.shape[0] / 3)
    # the reference's to_image((255 * (b / 256.0)).astype(uint8)) conversion, per texel
    bytes_in = (255 * (cross_u8[..., :3] / 256.0)).astype(np.uint8)
    faces = {k: bytes_in[r * n:(r + 1) * n, c * n:(c + 1) * n] for k, (r, c) in _CROSS.items()}
    out = np.zeros((3 * n, 4 * n, 3), dtype=np.uint8)
    for name, layout in _LAYOUTS.items():
        canvas = np.zeros((3 * n, 3 * n, 3), dtype=np.uint8)
        for (r, c), (src, k) in layout.items():
            canvas[r * n:(r + 1) * n, c * n:(c + 1) * n] = np.rot90(faces[src], k=k)
        img = Image.fromarray(canvas, "RGB").filter(ImageFilter.GaussianBlur(radius=blur))
        r, c = _CROSS[name]
        out[r * n:(r + 1) * n, c * n:(c + 1) * n] = np.asarray(img)[n:2 * n, n:2 * n]
    # immutable texels, like an image decoded by PIL: the scene lowering hashes them only once
    return np.frombuffer(out.tobytes(), dtype=np.uint8).reshape(out.shape)


def blur_skybox(img_array, blur, cubemap):
    """Reference signature: float (u8/256) cross in, linear-sRGB float cross out."""
    u8 = np.round(np.asarray(img_array) * 256.0).astype(np.uint8)
    return sRGB_to_sRGB_linear(blur_skybox_u8(u8, blur, cubemap) / 256.0)
