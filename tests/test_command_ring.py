"""The TP tier's shared-memory command ring (aios_amd/parallel/ring.py) on the CPU: binary
encoding round trip (no pickling), wrap-around, back-pressure on a slow worker, and a real
multi-process fan-out of engine-call-shaped commands (grammar masks as raw bytes)."""
import multiprocessing as mp
import os

import pytest

from aios_amd.parallel.ring import CommandRing, decode, encode


def _rt(o):
    b = bytearray()
    encode(o, b)
    v, n = decode(bytes(b))
    assert n == len(b)
    return v


def test_encoding_roundtrip():
    cmd = ["decode", [[0, 1, 2], [5, 6, 7], [12, 12, 13], [0.7, 0.0, 1.5], [40, 0, 0], 0, b"\x00\xff" * 9, [1.0, 0.9, 1.0],
                      [2**63 - 1, 5, 1]]]
    assert _rt(cmd) == cmd
    assert _rt([None, True, False, "x", [], [[1], [2.5]], b""]) == [None, True, False, "x", [], [[1], [2.5]], b""]
    # fresh uint64 sampling seeds (above int64) as scalars and in int lists
    big = 2**64 - 5
    assert _rt(["sample_first", [12, 0.7, 40, 0.9, big, b""]]) == ["sample_first", [12, 0.7, 40, 0.9, big, b""]]
    assert _rt([[big, 3, -1]]) == [[big, 3, -1]]
    with pytest.raises(TypeError):
        _rt(object())
    with pytest.raises(ValueError):
        decode(b"Z")


def _worker(name, world, rank, q):
    r = CommandRing(world, name=name, worker=rank)
    got = []
    while True:
        m = r.recv()
        if m == "__exit__":
            break
        got.append(m)
    q.put((rank, len(got), got[-1] if got else None, sum(len(x[1]) for x in got)))
    r.close()


def test_fanout_wraps_and_backpressures():
    world = 3
    ring = CommandRing(world, cap=1 << 16)  # small: forces many wraps and full-ring waits
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(ring.name, world, r, q)) for r in range(1, world)]
    for p in ps:
        p.start()
    mask = os.urandom(16032)  # one 128k-vocab grammar-mask row
    n = 300
    for i in range(n):
        ring.send(["decode", [[i], [i + 1], mask if i % 3 == 0 else b""]])
    ring.send("__exit__")
    res = sorted(q.get(timeout=60) for _ in ps)
    for p in ps:
        p.join(30)
    ring.close()
    assert [r[1] for r in res] == [n, n]
    assert all(r[2] == ["decode", [[n - 1], [n], mask if (n - 1) % 3 == 0 else b""]] for r in res)
    assert not os.path.exists("/dev/shm/" + ring.name)


def _leader(world, q, hold):
    r = CommandRing(world)
    q.put(r.name)
    hold.wait(60)  # never sends: the test SIGKILLs this process


def test_worker_exits_when_leader_is_killed():
    """a SIGKILLed leader runs no shutdown, so recv() must notice and raise ConnectionError
    (the worker then exits and frees its shard) instead of polling forever"""
    import signal
    import time
    from multiprocessing import shared_memory

    ctx = mp.get_context("spawn")
    q, hold = ctx.Queue(), ctx.Event()
    p = ctx.Process(target=_leader, args=(2, q, hold))
    p.start()
    name = q.get(timeout=60)
    r = CommandRing(2, name=name, worker=1)
    assert r.leader_pid == p.pid and r.leader_alive()
    try:
        os.kill(p.pid, signal.SIGKILL)
        t0 = time.monotonic()
        with pytest.raises(ConnectionError):
            r.recv()  # the dead leader is a zombie until joined: still detected
        assert time.monotonic() - t0 < 5
    finally:
        r.close()
        p.join(10)
        try:
            shm = shared_memory.SharedMemory(name=name)
            shm.close()
            shm.unlink()
        except FileNotFoundError:
            pass
