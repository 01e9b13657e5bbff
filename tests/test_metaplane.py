"""R4 metadata plane: the native shared-memory ring (csrc/runtime/meta_ring.cpp) that carries rank 0's
step metadata to the TP workers -- order, wrap-around, several readers in other processes, back-pressure
when a reader lags a whole ring, close, oversized messages, and the worker -> rank 0 fault back-channel."""
import multiprocessing as mp
import os
import uuid

import numpy as np
import pytest

from symmetry_amd.runtime import _runtime


def _name():
    return f"/symm-test-{os.getpid()}-{uuid.uuid4().hex[:8]}"


def test_ring_order_and_wraparound_single_process():
    name = _name()
    w = _runtime.MetaRing(name, 256, 4, 1, True)
    r = _runtime.MetaRing(name, 0, 0, 1, False)
    w.unlink()
    for k in range(11):  # wraps the 4-slot ring several times
        w.push(np.arange(k, k + 5, dtype=np.int32))
        got = r.pop(0, 1.0)
        assert got.dtype == np.int32 and got.tolist() == list(range(k, k + 5))
    assert w.written == 11 and w.nslots == 4 and w.slot_bytes == 256


def test_ring_refuses_oversized_and_times_out():
    name = _name()
    w = _runtime.MetaRing(name, 64, 2, 1, True)
    w.unlink()
    with pytest.raises(ValueError):
        w.push(np.zeros(17, dtype=np.int32))  # 68 B > 64 B slot
    with pytest.raises(TimeoutError):
        w.pop(0, 0.01)  # nothing published
    w.push(np.zeros(2, dtype=np.int32))
    w.push(np.zeros(2, dtype=np.int32))
    with pytest.raises(RuntimeError):  # the reader is a whole ring behind
        w.push(np.zeros(2, dtype=np.int32), 0.05)


def _reader(name, idx, n, q):
    r = _runtime.MetaRing(name, 0, 0, 3, False)
    total = 0
    seen = 0
    while True:
        m = r.pop(idx, 30.0)
        if m is None:
            break
        assert m[0] == seen, (m[0], seen)  # in order, none skipped
        total += int(m.sum())
        seen += 1
    q.put((idx, seen, total))


def test_ring_three_reader_processes_backpressure_and_close():
    name = _name()
    w = _runtime.MetaRing(name, 4096, 8, 3, True)
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    procs = [ctx.Process(target=_reader, args=(name, i, 500, q)) for i in range(3)]
    for p in procs:
        p.start()
    expect = 0
    for k in range(500):  # 500 messages through an 8-slot ring: the writer waits for the slowest reader
        msg = np.full(1 + k % 300, k, dtype=np.int32)
        msg[0] = k
        expect += int(msg.sum())
        w.push(msg, 30.0)
    w.shut()
    res = sorted(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(30)
    w.unlink()
    assert [r[1] for r in res] == [500] * 3
    assert all(r[2] == expect for r in res)


def test_ring_message_published_before_close_is_delivered():
    """A message pushed right before shut() is still delivered (pop re-checks the slot after seeing closed)."""
    name = _name()
    w = _runtime.MetaRing(name, 64, 4, 1, True)
    r = _runtime.MetaRing(name, 0, 0, 1, False)
    w.unlink()
    w.push(np.array([7, 8], dtype=np.int32))
    w.shut()
    assert r.pop(0, 1.0).tolist() == [7, 8]
    assert r.pop(0, 1.0) is None


def _failing_worker(name):
    r = _runtime.MetaRing(name, 0, 0, 2, False)
    r.register_pid(1, os.getpid())
    r.report(1, 5)


def _sleeper(name, ev):
    r = _runtime.MetaRing(name, 0, 0, 2, False)
    r.register_pid(0, os.getpid())
    ev.set()
    import time
    time.sleep(60)


def test_ring_faults_report_and_dead_reader():
    """faults(): a worker's reported code, and -1 for a registered reader whose process is gone."""
    name = _name()
    w = _runtime.MetaRing(name, 64, 2, 2, True)
    w.register_pid(-1, os.getpid())
    assert w.faults() == []
    ctx = mp.get_context("fork")
    ev = ctx.Event()
    sl = ctx.Process(target=_sleeper, args=(name, ev))
    sl.start()
    assert ev.wait(30)
    fw = ctx.Process(target=_failing_worker, args=(name,))
    fw.start()
    fw.join(30)
    assert w.faults() == [(1, 5)]
    sl.kill()  # SIGKILL: no chance to report
    sl.join(30)
    assert sorted(w.faults()) == [(0, -1), (1, 5)]
    # a push blocked on the dead reader fails fast instead of waiting out its timeout
    w.push(np.zeros(1, dtype=np.int32))
    w.push(np.zeros(1, dtype=np.int32))
    with pytest.raises(RuntimeError, match="failed"):
        w.push(np.zeros(1, dtype=np.int32), 30.0)
    w.unlink()
