"""The test-only RCCL stand-in (tests/stub_rccl.cpp) on the CPU, in its dry mode (host buffers, no
HIP call): the matching rules the world > 1 tiles GPU test relies on (tests/stub_tiles_worker.py).

* a root posting one receive per peer in one group and peers each posting a send, on separate
  threads (as the ranks of the GPU test run), receive exactly the peers' bytes, in any posting order;
* a loopback group (send to and receive from itself) completes alone;
* several sends between one pair match the receives in posting order (RTX_TILES_ROWS posts one per
  row block);
* differing sizes fail (ncclInvalidUsage), an unmatched operation times out (ncclInternalError)
  instead of hanging, and the log records every operation with its peer, bytes and address.
"""

import ctypes
import threading

import pytest

from python_ray_tracer_amd import _build

NCCL_UINT8 = 1
NCCL_FLOAT32 = 7


class UniqueId(ctypes.Structure):  # ncclUniqueId, passed by value
    _fields_ = [("internal", ctypes.c_char * 128)]


@pytest.fixture(scope="module")
def stub():
    try:
        path = _build.build_test_stub()
    except (FileNotFoundError, OSError) as e:  # pragma: no cover - no hipcc
        pytest.skip(f"cannot build the stub: {e}")
    lib = ctypes.CDLL(str(path))
    lib.ncclSend.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                             ctypes.c_void_p]
    lib.ncclRecv.argtypes = lib.ncclSend.argtypes
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, UniqueId, ctypes.c_int]
    lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
    lib.ncclGetErrorString.restype = ctypes.c_char_p
    lib.stub_rccl_log.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.stub_rccl_set_dry(1)
    lib.stub_rccl_set_timeout_ms(5000)
    return lib


def comms(lib, world):
    uid = UniqueId()
    assert lib.ncclGetUniqueId(ctypes.byref(uid)) == 0
    out = []
    for r in range(world):
        c = ctypes.c_void_p()
        assert lib.ncclCommInitRank(ctypes.byref(c), world, uid, r) == 0
        out.append(c)
    return out


def log(lib):
    n = lib.stub_rccl_log(None, 0)
    buf = (ctypes.c_longlong * (8 * max(n, 1)))()
    lib.stub_rccl_log(buf, n)
    keys = ("comm", "kind", "rank", "peer", "bytes", "ptr", "group", "seq")
    return [dict(zip(keys, buf[8 * i:8 * i + 8])) for i in range(n)]


def run_threads(fns):
    res = [None] * len(fns)

    def wrap(i):
        res[i] = fns[i]()
    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=30)
    assert not any(t.is_alive() for t in ts)
    return res


@pytest.mark.parametrize("root_first", [True, False])
def test_gather_to_root(stub, root_first):
    world, part = 4, 48
    cs = comms(stub, world)
    stub.stub_rccl_reset()
    recv = (ctypes.c_uint8 * (world * part))()
    sends = [(ctypes.c_uint8 * part)(*[(17 * r + i) % 251 for i in range(part)]) for r in range(world)]
    base = ctypes.addressof(recv)

    def root():
        assert stub.ncclGroupStart() == 0
        for p in range(1, world):
            assert stub.ncclRecv(base + p * part, part, NCCL_UINT8, p, cs[0], None) == 0
        return stub.ncclGroupEnd()

    def peer(r):
        def f():
            assert stub.ncclGroupStart() == 0
            assert stub.ncclSend(ctypes.addressof(sends[r]), part, NCCL_UINT8, 0, cs[r], None) == 0
            return stub.ncclGroupEnd()
        return f
    fns = [root] + [peer(r) for r in range(1, world)]
    if not root_first:
        fns = fns[::-1]
    assert run_threads(fns) == [0] * world
    got = bytes(recv)
    for p in range(1, world):
        assert got[p * part:(p + 1) * part] == bytes(sends[p])
    assert got[:part] == bytes(part)  # the root's own slot is left alone
    recs = log(stub)
    assert len(recs) == 2 * (world - 1)
    rx = sorted((r["peer"], r["bytes"], r["ptr"] - base) for r in recs if r["kind"] == 1)
    assert rx == [(p, part, p * part) for p in range(1, world)]
    tx = sorted((r["rank"], r["peer"], r["bytes"]) for r in recs if r["kind"] == 0)
    assert tx == [(r, 0, part) for r in range(1, world)]
    assert stub.stub_rccl_pending() == 0
    for c in cs:
        stub.ncclCommDestroy(c)


def test_loopback_group_and_pair_order(stub):
    (c,) = comms(stub, 1)
    src = (ctypes.c_float * 6)(*range(6))
    dst = (ctypes.c_float * 6)()
    assert stub.ncclGroupStart() == 0
    assert stub.ncclSend(ctypes.addressof(src), 6, NCCL_FLOAT32, 0, c, None) == 0
    assert stub.ncclRecv(ctypes.addressof(dst), 6, NCCL_FLOAT32, 0, c, None) == 0
    assert stub.ncclGroupEnd() == 0
    assert list(dst) == list(src)
    # several sends of one pair (one per row block) meet the receives in posting order
    a, b = comms(stub, 2)
    blocks = [(ctypes.c_uint8 * (3 + k))(*([k + 1] * (3 + k))) for k in range(4)]
    outs = [(ctypes.c_uint8 * (3 + k))() for k in range(4)]

    def sender():
        stub.ncclGroupStart()
        for blk in blocks:
            stub.ncclSend(ctypes.addressof(blk), len(blk), NCCL_UINT8, 0, b, None)
        return stub.ncclGroupEnd()

    def receiver():
        stub.ncclGroupStart()
        for o in outs:
            stub.ncclRecv(ctypes.addressof(o), len(o), NCCL_UINT8, 1, a, None)
        return stub.ncclGroupEnd()
    assert run_threads([receiver, sender]) == [0, 0]
    assert [bytes(o) for o in outs] == [bytes(blk) for blk in blocks]


def test_size_mismatch_and_unmatched(stub):
    a, b = comms(stub, 2)
    x = (ctypes.c_uint8 * 8)()
    y = (ctypes.c_uint8 * 16)()

    def s():
        return stub.ncclSend(ctypes.addressof(x), 8, NCCL_UINT8, 0, b, None)

    def r():
        return stub.ncclRecv(ctypes.addressof(y), 16, NCCL_UINT8, 1, a, None)
    rc = run_threads([s, r])
    assert rc == [5, 5], rc  # ncclInvalidUsage on both sides
    assert b"sizes differ" in stub.ncclGetErrorString(5)
    stub.stub_rccl_set_timeout_ms(200)
    try:
        assert stub.ncclSend(ctypes.addressof(x), 8, NCCL_UINT8, 0, b, None) == 3  # ncclInternalError
    finally:
        stub.stub_rccl_set_timeout_ms(5000)
    assert stub.stub_rccl_pending() == 0
    # a peer outside the communicator is refused at once
    assert stub.ncclSend(ctypes.addressof(x), 8, NCCL_UINT8, 2, b, None) == 4
