"""numpy's legacy `np.random.rand` stream reproduced by the segmented MT19937 jump-ahead scheme
(python-raytracer_amd/csrc/rt_mt.h, tables from tools/gen_mt_jump.py).  The oracle is numpy itself
(the stream the reference draws its camera jitter from: camera.py:51-85, utils/random.py:6-9); the
CPU tests run the scheme serially through the host-check build, the GPU tests run the HIP kernel
through the C ABI.  Bar: bit-exact doubles and an identical final numpy state."""
import sys

import numpy as np
import pytest

import hostcheck as HC
from conftest import ROOT

L_DOUBLES = (1 << 19) // 2  # doubles per device segment


def numpy_case(seed, pre, n_out, n_skip):
    rs = np.random.RandomState(seed)
    rs.random_sample(pre)
    st = rs.get_state()
    want = rs.random_sample(n_out)
    rs.random_sample(n_skip)
    end = rs.get_state()
    return st, want, end


CASES = [
    # seed, doubles drawn before (sets pos), n_out, n_skip
    (0, 0, 1000, 0),             # fresh seed: pos = 624
    (1, 1, 4097, 3),             # odd position
    (2, 311, 10, 0),             # pos = 622: first pair straddles a regeneration
    (3, 312, 1, 0),              # pos = 624 after draws
    (4, 5, 2 * L_DOUBLES + 17, 100),   # three segments (jumps x^(L-1), x^(2L-1))
    (5, 100, L_DOUBLES - 1, 2),  # ends right at a segment boundary
    (6, 7, 100, 17 * L_DOUBLES),  # skipped draws cross 17 segments
    (7, 3, 256 * L_DOUBLES + 1000, 5),  # outputs cross a round (256 segments): chained key window
    (8, 620, 40, 256 * L_DOUBLES - 45),  # final state window lands in the previous round
]


@pytest.mark.parametrize("seed,pre,n_out,n_skip", CASES)
def test_mt_segments_match_numpy_cpu(seed, pre, n_out, n_skip):
    st, want, end = numpy_case(seed, pre, n_out, n_skip)
    got, key, pos = HC.mt_uniforms(st[1], st[2], n_out, n_skip)
    assert np.array_equal(got, want)
    assert pos == end[2] and np.array_equal(key, end[1])


def test_jump_table_is_the_mt19937_jump():
    """Re-derive two table entries independently (pure Python MT words) and compare."""
    sys.path.insert(0, str(ROOT / "tools"))
    import gen_mt_jump as G

    src = (ROOT / "python-raytracer_amd" / "csrc" / "rt_mt_jump.h").read_text()
    import re

    body = src.split("static const uint32_t RT_MT_JD")[1].split("};")[0]
    rows = re.findall(r"\{(0x[^{}]*)\}", body)
    assert len(rows) == 255
    jd = [sum(int(v, 16) << (32 * k) for k, v in enumerate(r.split(","))) for r in (rows[0], rows[1])]
    G.check_jump(jd[0], G.L - 1)
    # consecutive entries differ by x^L: the second is x^(2L-1) (checked by its window)
    G.check_jump(jd[1], 2 * G.L - 1)


def _device_uniforms(st, n_out, n_skip, device_out=False):
    import ctypes
    from sightpy import _backend as B, _native as N

    np.random.set_state(st)
    if device_out:
        lib, ctx = B.context()
        p = B.numpy_uniforms(n_out, n_skip)
        got = np.empty(n_out)
        N.check(lib, lib.srt_memcpy(ctx, N.ptr(got), p, 8 * n_out))
    else:
        got = np.empty(n_out)
        B.numpy_uniforms(n_out, n_skip, out=got)
    return got, np.random.get_state()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,pre,n_out,n_skip", CASES)
def test_mt_device_matches_numpy(seed, pre, n_out, n_skip):
    st, want, end = numpy_case(seed, pre, n_out, n_skip)
    got, after = _device_uniforms(st, n_out, n_skip)
    assert np.array_equal(got, want)
    assert after[2] == end[2] and np.array_equal(after[1], end[1])


@pytest.mark.gpu
def test_mt_device_1080p_jitter_stream():
    """The parity-mode draw of Scene.render at the headline config (6 spp + the sizing draw at
    1920x1080), generated into device memory, equals numpy's stream."""
    npix = 1920 * 1080
    st, want, end = numpy_case(0, 0, 6 * 4 * npix, 4 * npix)
    got, after = _device_uniforms(st, 6 * 4 * npix, 4 * npix, device_out=True)
    assert np.array_equal(got, want)
    assert after[2] == end[2] and np.array_equal(after[1], end[1])


@pytest.mark.gpu
@pytest.mark.parametrize("parts", [2, 4, 8])
def test_mt_device_jump_parts_give_the_same_stream(parts):
    """Each jump window is XOR-accumulated by `parts` blocks over slices of the coefficient words
    (option mt_jump_parts): every split gives numpy's stream and final state."""
    from sightpy import _backend as B, _native as N

    lib, ctx = B.context()
    N.check(lib, lib.srt_set_option(ctx, b"mt_jump_parts", parts))
    try:
        st, want, end = numpy_case(11, 17, 3_000_001, 7)
        got, after = _device_uniforms(st, 3_000_001, 7)
        assert np.array_equal(got, want)
        assert after[2] == end[2] and np.array_equal(after[1], end[1])
    finally:
        N.check(lib, lib.srt_set_option(ctx, b"mt_jump_parts", 0))
    assert lib.srt_set_option(ctx, b"mt_jump_parts", 1) != 0


@pytest.mark.gpu
def test_scene_render_device_stream_equals_host_stream():
    import scenes

    sc = scenes.example1(160, 120, 3)
    np.random.seed(5)
    a = np.asarray(sc.render(2, rng="numpy"))
    sa = np.random.get_state()
    np.random.seed(5)
    b = np.asarray(sc.render(2, rng="numpy-host"))
    sb = np.random.get_state()
    # same jitter, and the framebuffer sums are order-independent: the same image
    assert np.array_equal(a, b)
    assert sa[2] == sb[2] and np.array_equal(sa[1], sb[1])


def test_host_jump_polynomials():
    """rt_mt.h xpow_mod (square-and-shift modulo the sparse phi) reproduces the tabulated jumps
    x^(sL - 1), and a jump by x^J lands on the window J words ahead of numpy's generator (the frame-end
    jump that lets pipelined frames start their stream before the previous frame's is generated)."""
    import re

    src = (ROOT / "python-raytracer_amd" / "csrc" / "rt_mt_jump.h").read_text()
    body = src.split("static const uint32_t RT_MT_JD")[1].split("};")[0]
    rows = re.findall(r"\{(0x[^{}]*)\}", body)
    for s in (1, 2, 200):
        want = np.array([int(v, 16) for v in rows[s - 1].split(",")], dtype=np.uint32)
        assert np.array_equal(HC.xpow_mod(s * (1 << 19) - 1), want)
    rs = np.random.RandomState(11)
    key = rs.get_state()[1]
    for J in (623, 5000, 3 * 624 * 1000 + 17):
        got = HC.jump_window(key, J)
        # numpy's raw words J .. J + 623 after the key window (words 0..623): regenerate with pure Python
        sys.path.insert(0, str(ROOT / "tools"))
        import gen_mt_jump as G

        words = G.raw_words([int(v) for v in key], J + 624)
        assert np.array_equal(got[1:], np.array(words[J + 1:J + 624], dtype=np.uint32))


def _mt_residue():
    import ctypes
    from sightpy import _backend as B, _native as N

    lib, ctx = B.context()
    nz = ctypes.c_int64(-1)
    N.check(lib, lib.srt_debug_mt_residue(ctx, ctypes.byref(nz)))
    return nz.value


@pytest.mark.gpu
def test_generator_state_is_clean_between_frames_of_changing_shapes():
    """Every generation leaves the segment-window tables, the end accumulator and its counter zero (the
    next generation's jump parts XOR into them): synchronous whole frames (short segments, band mode),
    pipelined frames (tabulated segments, frame-end jumps), a row shard (band mode), another frame
    shape, and the tabulated segments for a synchronous frame (mt_short=0)."""
    import ctypes
    import scenes
    from sightpy import _backend as B, _native as N

    lib, ctx = B.context()
    sc = scenes.example1(320, 240, 3)
    np.random.seed(3)
    B.render_scene(sc, 2, seed=1, mt=True)
    assert _mt_residue() == 0
    B.upload(sc)
    cd = B.camera_desc(sc.camera)
    mt = N.MtState.from_numpy()
    a = N.RenderArgs()
    a.spp, a.sample_base, a.n_rows, a.batch_spp = 2, 0, 240, 0
    a.rows, a.jitter, a.out_hit_id, a.seed = None, None, None, 1
    a.mt = ctypes.pointer(mt)
    a.flags = N.RENDER_ASYNC | N.RENDER_RGB_LOCAL
    u8 = [B.device_buffer("residue_u8_%d" % k, 3 * 320 * 240) for k in range(4)]
    for k in range(4):
        a.out_srgb8, a.out_rgb = u8[k], None
        N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), None))
    N.check(lib, lib.srt_render_finish(ctx, None))
    mt.to_numpy()
    assert _mt_residue() == 0
    rows = np.arange(5, 240, 3)
    B.render_scene(sc, 2, seed=1, mt=True, rows=rows)
    assert _mt_residue() == 0
    B.render_scene(scenes.example1(200, 150, 3), 3, seed=1, mt=True)
    assert _mt_residue() == 0
    N.check(lib, lib.srt_set_option(ctx, b"mt_short", 0))
    try:
        B.render_scene(sc, 2, seed=1, mt=True)
        assert _mt_residue() == 0
    finally:
        N.check(lib, lib.srt_set_option(ctx, b"mt_short", 65536))


@pytest.mark.gpu
def test_short_segment_frames_equal_tabulated_segment_frames():
    """A synchronous frame's numpy stream in short segments (band mode, option mt_short) and in the
    tabulated 2^19-word segments: the same image and the same numpy state afterwards (1080p, the
    headline's draw)."""
    import scenes
    from sightpy import _backend as B, _native as N

    lib, ctx = B.context()
    sc = scenes.example1(1920, 1080, 3)
    np.random.seed(11)
    a = B.render_scene(sc, 2, seed=1, mt=True)
    sa = np.random.get_state()
    N.check(lib, lib.srt_set_option(ctx, b"mt_short", 0))
    try:
        np.random.seed(11)
        b = B.render_scene(sc, 2, seed=1, mt=True)
        sb = np.random.get_state()
    finally:
        N.check(lib, lib.srt_set_option(ctx, b"mt_short", 65536))
    assert np.array_equal(a.rgb, b.rgb) and np.array_equal(a.srgb8, b.srgb8)
    assert sa[2] == sb[2] and np.array_equal(sa[1], sb[1])


@pytest.mark.gpu
def test_generator_width_gives_the_same_frames():
    """Pipelined frames of the lean fused kernel generate numpy's stream with four-wave generator
    workgroups (one wave per SIMD beside the trace waves; option mt_gen_nt auto = 256), other frames with
    five-wave ones: both widths give the same images and numpy state, whole frames and a shard's rows."""
    import ctypes

    import scenes
    from sightpy import _backend as B, _native as N

    lib, ctx = B.context()
    sc = scenes.example1(640, 360, 3)
    rows = [r for r in range(360) if (r // 9) % 8 == 3]

    def frames():
        np.random.seed(23)
        cd = B.camera_desc(sc.camera)
        out = []
        for rr in (None, rows):
            a = N.RenderArgs()
            n = 360 if rr is None else len(rr)
            ra = None if rr is None else np.ascontiguousarray(rr, dtype=np.int32)
            a.spp, a.sample_base, a.n_rows, a.batch_spp = 2, 0, n, 0
            a.rows, a.jitter, a.out_hit_id, a.out_rgb, a.seed = N.ptr(ra), None, None, None, 1
            mt = N.MtState.from_numpy()
            a.mt = ctypes.pointer(mt)
            a.flags = N.RENDER_ASYNC
            bufs = [B.pinned_buffer("width_u8_%d_%d" % (n, k), 3 * 640 * n) for k in range(3)]
            for k in range(3):
                a.out_srgb8 = N.ptr(bufs[k])
                N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), None))
            N.check(lib, lib.srt_render_finish(ctx, None))
            mt.to_numpy()
            out += [b.copy() for b in bufs]
        return out, np.random.get_state()

    try:
        N.check(lib, lib.srt_set_option(ctx, b"mt_gen_nt", 0))
        auto, sa = frames()
        N.check(lib, lib.srt_set_option(ctx, b"mt_gen_nt", 320))
        five, sb = frames()
    finally:
        N.check(lib, lib.srt_set_option(ctx, b"mt_gen_nt", 0))
    for x, y in zip(auto, five):
        assert np.array_equal(x, y)
    assert sa[2] == sb[2] and np.array_equal(sa[1], sb[1])
    assert lib.srt_set_option(ctx, b"mt_gen_nt", 100) != 0


@pytest.mark.gpu
@pytest.mark.parametrize("split", [0, 65536, 262144])
def test_pipelined_frames_segment_length_gives_the_same_frames(split):
    """Pipelined whole frames behind others in flight generate numpy's stream in band-mode segments of
    mt_pipe_split doubles (0: the tabulated 2^19-word segments): the same images and numpy state for
    every split, thin-lens camera (all four planes) included."""
    import ctypes

    import scenes
    from sightpy import _backend as B, _native as N

    lib, ctx = B.context()
    sc = scenes.example1(640, 360, 3)

    def frames(lens):
        sc.camera.lens_radius = lens
        np.random.seed(41)
        cd = B.camera_desc(sc.camera)
        a = N.RenderArgs()
        a.spp, a.sample_base, a.n_rows, a.batch_spp = 2, 0, 360, 0
        a.rows, a.jitter, a.out_hit_id, a.out_rgb, a.seed = None, None, None, None, 1
        mt = N.MtState.from_numpy()
        a.mt = ctypes.pointer(mt)
        a.flags = N.RENDER_ASYNC
        bufs = [B.pinned_buffer("split_u8_%d" % k, 3 * 640 * 360) for k in range(4)]
        for k in range(4):
            a.out_srgb8 = N.ptr(bufs[k])
            N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), None))
        N.check(lib, lib.srt_render_finish(ctx, None))
        mt.to_numpy()
        return [b.copy() for b in bufs], np.random.get_state()

    lens0 = sc.camera.lens_radius
    try:
        N.check(lib, lib.srt_set_option(ctx, b"mt_pipe_split", 0))
        ref = [frames(0.0), frames(0.05)]
        N.check(lib, lib.srt_set_option(ctx, b"mt_pipe_split", split))
        got = [frames(0.0), frames(0.05)]
    finally:
        N.check(lib, lib.srt_set_option(ctx, b"mt_pipe_split", 262144))
        sc.camera.lens_radius = lens0
    for (ra, sa), (rb, sb) in zip(ref, got):
        for x, y in zip(ra, rb):
            assert np.array_equal(x, y)
        assert sa[2] == sb[2] and np.array_equal(sa[1], sb[1])
