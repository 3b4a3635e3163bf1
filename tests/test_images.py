"""Host-side image plumbing of Scene.render (no GPU): the RGB image built over 4-byte pixels equals
the reference's Image.fromarray(..., "RGB") (reference scene.py:134-140), mapped or copied, and a
mapped image is read-only -- PIL copies it before any change, so the pixels it maps are never
written through it."""
import gc

import numpy as np
from PIL import Image

from sightpy import _backend as B


def _pixels(w, h, seed=0):
    rng = np.random.default_rng(seed)
    rgb = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    rgbx = np.concatenate([rgb, np.full((h, w, 1), 255, np.uint8)], axis=2)
    return rgb, np.ascontiguousarray(rgbx)


def test_rgb_image_equals_fromarray_mapped_and_copied():
    for w, h in ((1, 1), (7, 3), (160, 90), (1920, 1080)):
        rgb, rgbx = _pixels(w, h)
        ref = Image.fromarray(rgb, "RGB")
        for mapped in (True, False):
            img = B.rgb_image(rgbx, w, h, mapped)
            assert img.mode == "RGB" and img.size == (w, h)
            assert img.tobytes() == ref.tobytes()
            assert np.array_equal(np.asarray(img), rgb)


def test_mapped_image_is_copied_before_a_change_and_keeps_its_buffer_alive():
    rgb, rgbx = _pixels(32, 16, 1)
    keep = rgbx.copy()
    img = B.rgb_image(rgbx, 32, 16, True)
    img.putpixel((0, 0), (1, 2, 3))
    assert img.getpixel((0, 0)) == (1, 2, 3)
    assert np.array_equal(rgbx, keep)  # the mapped pixels were not written
    rgb2, rgbx2 = _pixels(8, 8, 2)
    img2 = B.rgb_image(rgbx2, 8, 8, True)
    del rgbx2
    gc.collect()
    assert np.array_equal(np.asarray(img2), rgb2)
    img2.save(__import__("io").BytesIO(), format="PNG")


def test_host_block_array_keeps_its_block_until_the_last_view_is_gone():
    released = []

    class Probe(B._HostBlock):
        __slots__ = ()

        def __del__(self):
            released.append(self.ptr)

    store = np.zeros(64, np.uint8)
    arr = np.asarray(Probe(store.ctypes.data, 64))
    assert arr.shape == (64,) and arr.dtype == np.uint8
    arr[:4] = (9, 8, 7, 6)
    assert list(store[:4]) == [9, 8, 7, 6]
    view = arr.reshape(8, 8)
    del arr
    gc.collect()
    assert not released
    img = B.rgb_image(view.reshape(4, 4, 4), 4, 4, True)
    del view
    gc.collect()
    assert not released  # the image maps it
    del img
    gc.collect()
    assert released == [store.ctypes.data]
