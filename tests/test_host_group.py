"""The cross-process host-staged collective backend (neus2_amd/csrc/hostgroup.h; include/neus2_hip.h neus_host_group_*)
on the CPU: world 2 and 3 processes over loopback TCP run the group's protocol on host buffers (neus_debug_host_group_
allreduce, no GPU) - f32 sums equal numpy's rank-order float32 sums bitwise (the in-process group's order), u32 sums and
f32 max exact - and ranks that issue different collectives fail loudly on every rank instead of pairing wrong buffers; a
connection with another job token is dropped while the real ranks join."""
import ctypes as C
import multiprocessing as mp
import socket
import struct
import time

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(rank, n, kind):
    rng = np.random.default_rng(100 + rank)
    if kind == "u32":
        return rng.integers(0, 1 << 20, n).astype(np.uint32)
    return (rng.normal(0, 1, n) * 10.0 ** rng.integers(-3, 3, n)).astype(np.float32)


TOKEN = 0x5EED1234ABCD0042


def _rank_main(rank, world, port, q, mismatch):
    try:
        from neus2_amd._lib import check, lib
        g = C.c_void_p()
        check(lib().neus_host_group_create(C.c_int(rank), C.c_int(world), b"127.0.0.1", C.c_int(port), C.c_uint64(TOKEN), C.byref(g)))
        out = {}
        try:
            for n, kind, op in ((1000, "f32", 0), (3, "u32", 0), (70000, "f32", 1), (1, "f32", 0)):
                x = _data(rank, n, kind)
                if mismatch and rank == 1:
                    x = x[:-1].copy() if n > 1 else x
                check(lib().neus_debug_host_group_allreduce(g, C.c_void_p(x.ctypes.data), C.c_uint64(x.size),
                                                             C.c_int(1 if kind == "u32" else 0), C.c_int(op)))
                out[(n, kind, op)] = x
            q.put((rank, "ok", out))
        except Exception as e:  # noqa: BLE001 - reported to the parent
            q.put((rank, "error", str(e)))
        finally:
            lib().neus_host_group_destroy(g)
    except Exception as e:  # noqa: BLE001
        q.put((rank, "error", "setup: " + str(e)))


def _intrude(port):
    """A foreign connection to rank 0 whose hello {magic, rank 1, token} carries another job token; returns the socket once
    rank 0 has closed it (recv sees EOF)."""
    t0 = time.time()
    while True:
        s = socket.socket()
        try:
            s.connect(("127.0.0.1", port))
            break
        except OSError:
            s.close()
            assert time.time() - t0 < 60, "rank 0 never listened"
            time.sleep(0.05)
    s.sendall(struct.pack("<IiQ", 0x4E484731, 1, TOKEN ^ 1))
    s.settimeout(30)
    assert s.recv(1) == b"", "rank 0 kept a connection with the wrong job token"
    return s


def _run(world, mismatch=False, intruder=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, q, mismatch)) for r in range(world)]
    if intruder:  # rank 0 first; the foreign hello is dropped before the real ranks start
        ps[0].start()
        _intrude(port).close()
        for p in ps[1:]:
            p.start()
    else:
        for p in ps:
            p.start()
    res = {}
    for _ in range(world):
        r, status, payload = q.get(timeout=180)
        res[r] = (status, payload)
    for p in ps:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_host_group_allreduce_matches_rank_order_sums(world):
    res = _run(world)
    for r in range(world):
        assert res[r][0] == "ok", res[r]
    for (n, kind, op), got0 in res[0][1].items():
        parts = [_data(r, n, kind) for r in range(world)]
        if op == 1:
            ref = parts[0].copy()
            for v in parts[1:]:
                ref = np.maximum(ref, v)
        else:
            ref = parts[0].copy()
            for v in parts[1:]:
                ref = (ref + v).astype(ref.dtype)  # rank order, one rounding per rank (NeusLocalGroup's order)
        for r in range(world):
            np.testing.assert_array_equal(res[r][1][(n, kind, op)].view(np.uint32), ref.view(np.uint32))


def test_host_group_mismatched_collectives_fail_on_every_rank():
    res = _run(2, mismatch=True)
    assert res[0][0] == "error" and "different collective" in res[0][1], res[0]
    assert res[1][0] == "error", res[1]


def test_host_group_drops_a_connection_with_another_job_token():
    res = _run(2, intruder=True)
    assert res[0][0] == "ok" and res[1][0] == "ok", res
