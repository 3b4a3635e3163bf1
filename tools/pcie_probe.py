"""Device -> pinned host copy rate through the library (srt_host_alloc + srt_memcpy), with the NUMA
node of the GPU and of the calling CPU: a host-inclusive frame streams its linear RGB over PCIe, so
this rate bounds it (python tools/pcie_probe.py [MB])."""
import ctypes
import glob
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "python-raytracer_amd"))
from sightpy import _backend as B, _native as N  # noqa: E402


def gpu_numa_nodes():
    out = []
    for card in sorted(glob.glob("/sys/class/drm/card*/device/numa_node")):
        try:
            out.append((card.split("/")[4], int(open(card).read().strip())))
        except (OSError, ValueError):
            pass
    return out


def main():
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    lib, ctx = B.context()
    n = mb << 20
    dev, host = ctypes.c_void_p(), ctypes.c_void_p()
    N.check(lib, lib.srt_device_alloc(ctx, n, ctypes.byref(dev)))
    N.check(lib, lib.srt_host_alloc(ctx, n, ctypes.byref(host)))
    # NUMA node of the buffer's first page (move_pages query)
    libc = ctypes.CDLL(None, use_errno=True)
    pages = (ctypes.c_void_p * 1)(host.value)
    status = (ctypes.c_int * 1)(-99)
    libc.syscall(279, 0, 1, pages, None, status, 0)
    for _ in range(3):
        N.check(lib, lib.srt_memcpy(ctx, host, dev, n))
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        N.check(lib, lib.srt_memcpy(ctx, host, dev, n))
        ts.append(time.perf_counter() - t0)
    ts.sort()
    cpu = os.sched_getcpu() if hasattr(os, "sched_getcpu") else -1
    node = -1
    for d in glob.glob("/sys/devices/system/node/node*"):
        try:
            cpus = open(d + "/cpulist").read().strip()
        except OSError:
            continue
        for part in cpus.split(","):
            lo, _, hi = part.partition("-")
            if lo and int(lo) <= cpu <= int(hi or lo):
                node = int(d.rsplit("node", 1)[1])
    print("D2H pinned %d MB: median %.2f GB/s (best %.2f); buffer on node %d; cpu %d on node %d; GPU numa nodes %s; "
          "affinity %d cpus" % (mb, n / ts[len(ts) // 2] / 1e9, n / ts[0] / 1e9, status[0], cpu, node, gpu_numa_nodes()[:8],
             len(os.sched_getaffinity(0))), flush=True)
    lib.srt_host_free(ctx, host)
    lib.srt_device_free(ctx, dev)


if __name__ == "__main__":
    main()
