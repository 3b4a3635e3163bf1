"""A stand-in for libsightpy_hip.so's C ABI (include/sightpy_rt.h) in Python, for CPU tests of the
multi-GPU bench plumbing (tests/test_bench_n8.py): what bench.py hands to srt_render /
srt_render_group / the communicator entry points at N = 8, checked call by call.

It renders nothing.  A frame "writes" the linear-RGB rows the real library would write for the
caller (SRT_RENDER_RGB_ROWS: the rank's own row bands, sightpy._shard's partition, as value
owner + 1) so the test can check that the ranks' writes tile the shared host frame exactly; a
violated expectation returns SRT_ERR_ARG with the reason in srt_last_error, as the library's own
argument checks do.  Collectives across the ranks' processes go through files in `sync_dir`."""
import ctypes
import json
import os
import time

import numpy as np

from sightpy import _native as N
from sightpy._shard import shard_kmax, shard_rows

ERR = 2  # any nonzero rc: bench.py's N.check raises with srt_last_error()


def _obj(ref):
    """The object behind a ctypes.byref() argument."""
    return ref._obj if hasattr(ref, "_obj") else ref


class FakeSrt:
    def __init__(self, W, H, spp, world, rank, sync_dir, fanout=1, group=False):
        self.W, self.H, self.spp, self.world, self.rank = W, H, spp, world, rank
        self.sync_dir, self.group = sync_dir, group
        self.kmax = shard_kmax(H, world, 0, fanout)
        self.err = b""
        self.host = {}  # address -> (ctypes buffer, bytes) of srt_host_alloc
        self.registered = {}  # address -> bytes of srt_host_register
        self.options = {}
        self.frames = []  # (flags, async) per rendered frame
        self.ncoll = 0
        self.comm = None
        self.lean = 0
        self.lane = None
        self.rgb_rows_frames = set()  # addresses written with SRT_RENDER_RGB_ROWS
        self.log = {"rank": rank, "checks": []}

    # ---- helpers -------------------------------------------------------------------------------
    def fail(self, msg):
        self.err = msg.encode()
        self.log.setdefault("errors", []).append(msg)
        self._dump()
        return ERR

    def _dump(self):
        with open(os.path.join(self.sync_dir, "fake_rank%d.json" % self.rank), "w") as fh:
            json.dump(self.log, fh)

    def _rows(self, q):
        return shard_rows(self.H, self.world, q, self.kmax)

    def _stats(self, st, rays_scale=1):
        if st is None:
            return
        s = _obj(st)
        npix = len(self._rows(self.rank)) * self.W if self.world > 1 else self.W * self.H
        depth = [npix * self.spp, npix * self.spp // 2, npix * self.spp // 8]
        for d, v in enumerate(depth):
            s.rays_per_depth[d] = v * rays_scale
        s.n_depths = len(depth)
        s.total_rays = sum(depth) * rays_scale
        s.shadow_rays = depth[0] * rays_scale
        s.passes = 1
        s.ms_primary_kernel = 0.05
        s.ms_device = 0.06
        s.ms_wall = 0.07
        s.kernel_path = 2  # "fused": bench.py's lean-kernel roofline path runs too
        s.chain_from = 0

    def _collective(self, kind, payload):
        """Blocking exchange of `payload` with every rank (files in sync_dir)."""
        k = self.ncoll
        self.ncoll += 1
        me = os.path.join(self.sync_dir, "%s_%d_r%d.json" % (kind, k, self.rank))
        with open(me + ".tmp", "w") as fh:
            json.dump(payload, fh)
        os.replace(me + ".tmp", me)
        paths = [os.path.join(self.sync_dir, "%s_%d_r%d.json" % (kind, k, q)) for q in range(self.world)]
        t0 = time.time()
        while not all(os.path.exists(p) for p in paths):
            if time.time() - t0 > 120:
                raise RuntimeError("fake collective %s #%d: ranks missing" % (kind, k))
            time.sleep(0.005)
        return [json.load(open(p)) for p in paths]

    def _write_rows(self, addr, q):
        """rank q's rows of the [3][H*W] f64 host frame at addr := q + 1 (SRT_RENDER_RGB_ROWS)."""
        frame = np.ctypeslib.as_array((ctypes.c_double * (3 * self.W * self.H)).from_address(addr))
        fr = frame.reshape(3, self.H, self.W)
        fr[:, self._rows(q), :] = q + 1
        self.rgb_rows_frames.add(addr)

    def _check_frame(self, addr):
        fr = np.ctypeslib.as_array((ctypes.c_double * (3 * self.W * self.H)).from_address(addr)).reshape(
            3, self.H, self.W)
        want = np.empty(self.H)
        for q in range(self.world):
            want[self._rows(q)] = q + 1
        ok = bool(np.array_equal(fr, np.broadcast_to(want[None, :, None], fr.shape)))
        self.log["checks"].append({"frame": "rgb_rows", "tiled_exactly": ok})
        self._dump()
        return ok

    def _check_args(self, a, async_, where):
        if a.spp != self.spp or a.n_rows != self.H or a.rows:
            return "%s: spp/n_rows/rows %d/%d/%r" % (where, a.spp, a.n_rows, a.rows)
        if a.jitter or not a.mt:
            return "%s: the jitter must come from numpy's stream on the device (mt state given)" % where
        f = a.flags
        if bool(f & N.RENDER_ASYNC) != async_:
            return "%s: async flag %d" % (where, f)
        if f & N.RENDER_RGB_ROWS:
            if not async_ and self.group:
                return "%s: RGB_ROWS needs ASYNC in a group frame" % where
            if f & N.RENDER_RGB_LOCAL or not a.out_rgb:
                return "%s: RGB_ROWS with RGB_LOCAL or without out_rgb" % where
        elif f & N.RENDER_RGB_LOCAL:
            if a.out_rgb:
                return "%s: RGB_LOCAL with out_rgb" % where
        else:
            return "%s: neither RGB_ROWS nor RGB_LOCAL (flags %d)" % (where, f)
        return None

    # ---- the C ABI ----------------------------------------------------------------------------
    def srt_last_error(self):
        return self.err

    def srt_device_count(self, n):
        _obj(n).value = 8
        return 0

    def srt_create(self, dev, out):
        if dev != self.rank:
            return self.fail("rank %d created its context on device %d (LOCAL_RANK)" % (self.rank, dev))
        _obj(out).value = 0x1000 + dev
        return 0

    def srt_destroy(self, ctx):
        return 0

    def srt_set_option(self, ctx, key, value):
        self.options[key.decode()] = int(value.value if hasattr(value, "value") else value)
        return 0

    def srt_upload_scene(self, ctx, desc):
        self.log["uploads"] = self.log.get("uploads", 0) + 1
        return 0

    def srt_comm_unique_id(self, buf):
        if self.rank != 0:
            return self.fail("srt_comm_unique_id on rank %d" % self.rank)
        for i in range(N.COMM_ID_BYTES):
            buf[i] = (i * 7 + 3) & 255
        return 0

    def srt_comm_init(self, ctx, nranks, rank, cid):
        if (nranks, rank) != (self.world, self.rank):
            return self.fail("srt_comm_init(%d, %d) on rank %d of %d" % (nranks, rank, self.rank, self.world))
        if any(cid[i] != (i * 7 + 3) & 255 for i in range(N.COMM_ID_BYTES)):
            return self.fail("rank %d got another communicator id than rank 0 made" % self.rank)
        self.comm = (nranks, rank)
        return 0

    def srt_comm_init_all(self, n, devs, ctxs):
        if n != self.world or [devs[q] for q in range(n)] != list(range(n)):
            return self.fail("srt_comm_init_all over %r" % [devs[q] for q in range(n)])
        for q in range(n):
            ctxs[q] = 0x1000 + q
        self.comm = (n, 0)
        return 0

    def srt_comm_rank(self, ctx, nr, rk):
        n, r = self.comm if self.comm else (1, 0)
        _obj(nr).value, _obj(rk).value = n, r
        return 0

    def srt_comm_barrier(self, ctx):
        self._collective("bar", 0)
        return 0

    def srt_comm_allreduce(self, ctx, vals, n, op):
        got = self._collective("ar", [vals[i] for i in range(n)])
        for i in range(n):
            xs = [g[i] for g in got]
            vals[i] = sum(xs) if op == 0 else max(xs)
        return 0

    def srt_host_alloc(self, ctx, nbytes, out):
        buf = (ctypes.c_char * int(nbytes))()
        addr = ctypes.addressof(buf)
        self.host[addr] = (buf, int(nbytes))
        _obj(out).value = addr
        return 0

    def srt_host_free(self, ctx, p):
        addr = p.value if hasattr(p, "value") else p
        if addr in self.rgb_rows_frames:
            self._check_frame(addr)
        self.host.pop(addr, None)
        return 0

    def srt_host_register(self, ctx, p, nbytes):
        addr = p.value if hasattr(p, "value") else p
        if int(nbytes) != 3 * self.W * self.H * 8:
            return self.fail("registered %d bytes, the frame's RGB is %d" % (nbytes, 3 * self.W * self.H * 8))
        self.registered[addr] = int(nbytes)
        return 0

    def srt_host_unregister(self, ctx, p):
        addr = p.value if hasattr(p, "value") else p
        if self.rank == 0 and addr in self.rgb_rows_frames:
            self._check_frame(addr)  # (after bench.py's last barrier: every rank's rows are in)
        self.registered.pop(addr, None)
        return 0

    def srt_render(self, ctx, cd, a, st):
        a = _obj(a)
        async_ = bool(a.flags & N.RENDER_ASYNC)
        msg = self._check_args(a, async_, "srt_render rank %d" % self.rank)
        if msg:
            return self.fail(msg)
        if self.world > 1 and not a.flags & N.RENDER_SHARDED:
            return self.fail("a rank's frame without SRT_RENDER_SHARDED")
        if self.rank == 0:
            if not a.out_srgb8 or a.out_srgb8 not in self.host or self.host[a.out_srgb8][1] < 3 * self.W * self.H:
                return self.fail("rank 0's uint8 output is not a pinned whole-frame buffer")
        elif a.out_srgb8:
            return self.fail("rank %d passed a uint8 output (only rank 0 receives the gathered frame)" % self.rank)
        if a.flags & N.RENDER_RGB_ROWS:
            if os.environ.get("FAKE_SRT_FAIL_RGB_ROWS"):  # (injected failure: tests/test_bench_n8.py)
                return self.fail("injected: RGB_ROWS frame failed")
            if a.out_rgb not in self.registered:
                return self.fail("RGB_ROWS into memory not registered with srt_host_register")
            self._write_rows(a.out_rgb, self.rank)
        self.frames.append((int(a.flags), async_))
        self.log["frames"] = len(self.frames)
        if async_ or self.options.get("sync_lean"):
            self.lean += 1  # (the library's k_primary_lean launches: pipelined frames, or sync_lean)
        if self.lane is not None:
            self.lane += 1
        self._stats(st)
        self._dump()
        return 0

    def srt_render_finish(self, ctx, st):
        self._stats(st)
        return 0

    def srt_synchronize(self, ctx):
        return 0

    def srt_render_group(self, ctxs, n, cd, a, st):
        a = _obj(a)
        if n != self.world or len({ctxs[q] for q in range(n)}) != n:
            return self.fail("srt_render_group over %d contexts %r" % (n, [ctxs[q] for q in range(n)]))
        async_ = bool(a.flags & N.RENDER_ASYNC)
        msg = self._check_args(a, async_, "srt_render_group")
        if msg:
            return self.fail(msg)
        if a.flags & N.RENDER_SHARDED:
            return self.fail("srt_render_group sets SHARDED itself")
        if not a.out_srgb8 or a.out_srgb8 not in self.host:
            return self.fail("the group's uint8 output is not pinned host memory")
        if a.flags & N.RENDER_RGB_ROWS:
            if a.out_rgb not in self.host or self.host[a.out_rgb][1] != 3 * self.W * self.H * 8:
                return self.fail("RGB_ROWS into a buffer that is not the whole frame's pinned RGB")
            for q in range(n):
                self._write_rows(a.out_rgb, q)
        self.frames.append((int(a.flags), async_))
        self.log["frames"] = len(self.frames)
        self._stats(st, rays_scale=1)
        return 0

    def srt_render_group_finish(self, ctxs, n, st):
        self._stats(st)
        return 0

    def srt_debug_lean_launches(self, ctx, out):
        _obj(out).value = self.lean
        return 0

    def srt_debug_lane_stats(self, ctx, mode, out, n):
        if mode == 1:
            self.lane = 0
            return 0
        if self.lane is None:
            return self.fail("lane stats read before start")
        for d in range(n):
            out[2 * d] = 10 * self.lane if d < 3 else 0
            out[2 * d + 1] = 600 * self.lane if d < 3 else 0
        self.log["lane_frames"] = self.lane
        self.lane = None
        self._dump()
        return 0
