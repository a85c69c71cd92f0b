"""The loopback communicator of kg_place_sharded (koordinator_amd/csrc/kg_comm.cpp) on the CPU: world 2 and 8
processes all-reduce (max) random buffers many rounds in a row (the double-buffered slot sets: a fast rank must
not overwrite a slot a slow one still reads), sizes up to the slot, a rank that never arrives (timeout, no hang), an
aborting rank (its peers fail at their next wait), a world mismatch, and that nothing is left in /dev/shm."""
import ctypes
import multiprocessing as mp
import os
import subprocess
import time
import uuid

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "koordinator_amd", "csrc")
SHIM_DIR = os.path.join(ROOT, "build", "shm_shim")
SHIM_SO = os.path.join(SHIM_DIR, "libshmshim.so")


def _build():
    srcs = [os.path.join(CSRC, "kg_comm.cpp"), os.path.join(os.path.dirname(__file__), "shm_comm_shim.cpp")]
    os.makedirs(SHIM_DIR, exist_ok=True)
    if os.path.exists(SHIM_SO) and all(os.path.getmtime(s) < os.path.getmtime(SHIM_SO) for s in srcs):
        return SHIM_SO
    tmp = f"{SHIM_SO}.{os.getpid()}.tmp"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fPIC", "-shared", "-Wall", f"-I{CSRC}", *srcs, "-o", tmp,
                    "-lrt"], check=True)
    os.replace(tmp, SHIM_SO)
    return SHIM_SO


def _lib():
    L = ctypes.CDLL(_build())
    vp = ctypes.c_void_p
    L.shim_open.restype = vp
    L.shim_open.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_double]
    L.shim_allreduce.argtypes = [vp, vp, ctypes.c_size_t]
    L.shim_abort.argtypes = [vp]
    L.shim_close.argtypes = [vp]
    L.shim_error.restype = ctypes.c_char_p
    return L


def _rank_rounds(name, rank, world, rounds, count, q):
    try:
        L = _lib()
        c = L.shim_open(name.encode(), rank, world, count * 4, 30.0)
        if not c:
            q.put((rank, "open: " + L.shim_error().decode()))
            return
        rng = np.random.default_rng(1000 + rank)
        for r in range(rounds):
            n = int(np.random.default_rng(r).integers(1, count + 1))   # the same size on every rank, per round
            buf = (np.random.default_rng(r * 64 + rank).integers(0, 2**32, n, dtype=np.uint64)).astype(np.uint32)
            if rank == r % world:
                time.sleep(float(rng.random()) * 0.002)   # a different slow rank every round
            if L.shim_allreduce(c, buf.ctypes.data, n):
                q.put((rank, f"round {r}: " + L.shim_error().decode()))
                return
            want = np.max([np.random.default_rng(r * 64 + k).integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
                           for k in range(world)], axis=0)
            if not np.array_equal(buf, want):
                q.put((rank, f"round {r}: wrong max"))
                return
        L.shim_close(c)
        q.put((rank, "ok"))
    except Exception as ex:  # noqa: BLE001
        q.put((rank, repr(ex)))


def _run(world, target, *args, timeout=120):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/kgtest_{uuid.uuid4().hex[:12]}"
    ps = [ctx.Process(target=target, args=(name, r, world, *args, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    deadline = time.time() + timeout
    while len(out) < len(ps) and time.time() < deadline:
        try:
            r, msg = q.get(timeout=1.0)
            out[r] = msg
        except Exception:  # noqa: BLE001
            pass
    for p in ps:
        p.join(timeout=5)
        if p.is_alive():
            p.kill()
    assert not os.path.exists("/dev/shm" + name), "the segment must be unlinked (all joined, or the join failed)"
    return out


@pytest.mark.parametrize("world", [2, 8])
def test_allreduce_rounds(world):
    out = _run(world, _rank_rounds, 200, 4096)
    assert out == {r: "ok" for r in range(world)}, out


def _rank_absent(name, rank, world, q):
    L = _lib()
    if rank == world - 1:
        q.put((rank, "absent"))
        return
    t0 = time.time()
    c = L.shim_open(name.encode(), rank, world, 1024, 2.0)
    q.put((rank, ("open failed" if not c else "opened") + f" {time.time() - t0:.1f}"))


def test_absent_rank_times_out():
    out = _run(3, _rank_absent)
    for r in range(2):
        msg, t = out[r].rsplit(" ", 1)
        assert msg == "open failed" and 1.5 < float(t) < 20, out


def _rank_abort(name, rank, world, q):
    L = _lib()
    c = L.shim_open(name.encode(), rank, world, 1024, 30.0)
    buf = np.zeros(16, np.uint32)
    assert L.shim_allreduce(c, buf.ctypes.data, 16) == 0
    if rank == 0:
        L.shim_abort(c)
        q.put((rank, "aborted"))
        return
    t0 = time.time()
    st = L.shim_allreduce(c, buf.ctypes.data, 16)
    q.put((rank, f"{st} {time.time() - t0 < 10} {L.shim_error().decode()}"))


def test_abort_releases_peers():
    out = _run(4, _rank_abort)
    assert out[0] == "aborted"
    for r in range(1, 4):
        assert out[r].startswith("1 True") and "aborted" in out[r], out


def _rank_world(name, rank, world, q):
    L = _lib()
    c = L.shim_open(name.encode(), rank, world + rank, 1024, 3.0)   # rank 1 claims a different world
    q.put((rank, "opened" if c else L.shim_error().decode()))


def test_world_mismatch_refused():
    out = _run(2, _rank_world)
    assert any("world" in m for m in out.values()), out
