"""sRGB transfer functions (reference `utils/colour_functions.py:4-28`).

`sRGB_to_sRGB_linear` is used on the host to build the 256-entry per-texture lookup tables that
the kernels index with the raw texel byte (so a device texel fetch reproduces
`load_image_as_linear_sRGB` exactly).  The frame resolve (`sRGB_linear_to_sRGB` + clip + u8) of a
render runs on the device (`k_resolve` in `csrc/rt_kernels.hip`); these host versions remain part
of the public API.
"""
import numpy as np

__all__ = ["sRGB_linear_to_sRGB", "sRGB_to_sRGB_linear"]


def sRGB_linear_to_sRGB(rgb_linear):
    """Inverse gamma + per-pixel max-channel intensity clip, on a (3, ...) array."""
    encoded = np.where(
        rgb_linear <= 0.00304,
        12.92 * rgb_linear,
        1.055 * np.power(rgb_linear, 1.0 / 2.4) - 0.055,
    )
    peak = np.amax(encoded, axis=0) + 0.00001
    cutoff = 1.0
    return np.where(peak > cutoff, encoded * cutoff / peak, encoded)


def sRGB_to_sRGB_linear(rgb):
    """sRGB -> linear (reference `colour_functions.py:21-28`)."""
    return np.where(rgb <= 0.03928, rgb / 12.92, np.power((rgb + 0.055) / 1.055, 2.4))
