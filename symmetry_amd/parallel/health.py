"""TP fault containment on rank 0 (VERDICT r3 "Contain TP faults").

The reference keeps a provider alive and answering the server's ``ping`` (``src/provider.ts:124-126``) and
abandons a failed request without telling the client (``:270-274``).  A tensor-parallel provider whose
worker rank died can still answer pings but can no longer serve: every collective of every later step waits
for a peer that will never arrive.  So rank 0 watches its peers and, on the first fault:

1. declares it on the xGMI communicator (host-mapped error word): every spinning collective on the GPU stops
   waiting within a few polls (``csrc/kernels/xgmi_ar.hip``, ``xg_fault_declared``), so the step in flight
   finishes -- with garbage the host discards -- instead of costing one wait limit per collective;
2. calls its listeners once: the engine fails every request with an error output, the backend ends every
   open stream with the error SSE event + ``inferenceEnded``, and the provider sends ``leave`` to the server
   and exits non-zero, so a supervisor can start a fresh set of ranks (no re-exec here).

Faults come from three places: a worker's own report or its vanished process (the metadata ring's
back-channel, ``csrc/runtime/meta_ring.cpp``), and the xGMI error word (a collective that gave up waiting).
"""
from __future__ import annotations

import threading
import time


class TPFaultError(RuntimeError):
    """A step lost a tensor-parallel peer: neither it nor any later step can produce valid outputs."""


class TPHealthMonitor:
    def __init__(self, meta, comm=None, period_s: float = 0.1):
        self.meta = meta
        self.comm = comm
        self.period_s = period_s
        self.fault: str | None = None
        self._listeners: list = []
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    def add_listener(self, fn) -> None:
        """``fn(message)`` runs once, on the monitor thread (or at once if a fault is already known)."""
        with self._lock:
            fault = self.fault
            if fault is None:
                self._listeners.append(fn)
        if fault is not None:
            fn(fault)

    def check(self) -> str | None:
        """One poll: a description of the first fault seen, else None."""
        if self.fault is not None:
            return self.fault
        for rank, code in (self.meta.faults() if self.meta is not None else []):
            what = "exited" if code == -1 else f"reported failure code {code}"
            return self.declare(f"tensor-parallel rank {rank} {what}", 1 + rank)
        err = getattr(self.comm, "error", None)
        code = err() if err is not None else 0
        if code:
            return self.declare(f"xGMI collective gave up waiting for tensor-parallel rank {code - 1}", code)
        return None

    def declare(self, message: str, code: int = 1) -> str:
        """Record the fault (first one wins), stop the device collectives, notify the listeners."""
        with self._lock:
            if self.fault is not None:
                return self.fault
            self.fault = message
            listeners, self._listeners = self._listeners, []
        set_err = getattr(self.comm, "set_error", None)
        if set_err is not None:
            try:
                set_err(max(1, int(code)))
            except Exception:  # noqa: BLE001 -- a dying communicator must not mask the fault itself
                pass
        for fn in listeners:
            try:
                fn(message)
            except Exception:  # noqa: BLE001
                import traceback

                traceback.print_exc()
        return message

    def start(self) -> "TPHealthMonitor":
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="symmetry-tp-health", daemon=True)
            self._thread.start()
        return self

    def _run(self) -> None:
        while not self._stop.wait(self.period_s):
            try:
                if self.check() is not None:
                    return
            except Exception:  # noqa: BLE001 -- e.g. the ring was released at shutdown
                if self._stop.is_set():
                    return
                time.sleep(self.period_s)

    def stop(self) -> None:
        self._stop.set()
