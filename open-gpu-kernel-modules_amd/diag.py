"""Hang diagnostics for rank processes.

A multi-rank job that stops making progress must leave evidence: every rank's
Python stacks (all threads) and the runtime's own view - each ring's pushed /
submitted / completed tracking values, what its DMA worker is blocked on (a
fence, a stream drain) and for how long, the outstanding leases
(``lib.debug_dump``, try-locks only). The reference prints the push
description of the work a channel is stuck on (uvm_channel.c:2090-2100); this
is the user-space equivalent for a job of one process per GPU.

Two triggers, both handled on a dedicated daemon thread (the main thread may
be blocked inside the runtime or a collective and never return to the
interpreter, so an ordinary Python signal handler would never run):

  * ``SIGUSR1`` - the launcher (bench.py) sends it to every rank before it
    kills a job that outlived its timeout;
  * a watchdog deadline (``arm(seconds, what)``) - for launchers that do not
    signal (torchrun): the rank dumps itself once if the armed phase overruns.

``install()`` must run before any other thread exists (first thing in a rank,
before torch starts its threads): SIGUSR1 is blocked in the calling thread, so
every thread created later inherits the mask and only the dump thread takes
the signal (``sigwait``); the default action - terminate - can never hit.
"""
from __future__ import annotations

import faulthandler
import os
import signal
import sys
import threading
import time
from typing import Optional

_installed = False
_lock = threading.Lock()
_deadline: Optional[float] = None
_what = ""
_tag = ""
_dumps = 0


def _native_dump() -> str:
    try:
        from ._native import lib
        return lib.debug_dump()
    except Exception as e:  # noqa: BLE001 - diagnostics must never raise
        return f"[ogkm-dump] native dump unavailable: {type(e).__name__}: {e}\n"


def dump(reason: str, stream=None) -> None:
    """Write every thread's Python stack and the runtime state to ``stream``
    (stderr) as one block: assembled in a temporary file first, then written at
    once, staggered by local rank, so the dumps of ranks sharing the launcher's
    stderr do not interleave."""
    import tempfile
    global _dumps
    out = stream or sys.stderr
    with _lock:
        _dumps += 1
        try:
            with tempfile.TemporaryFile(mode="w+") as tf:
                tf.write(f"\n[ogkm-hang] {_tag}pid {os.getpid()}: {reason}\n")
                tf.flush()
                faulthandler.dump_traceback(file=tf, all_threads=True)
                tf.write(_native_dump())
                tf.write(f"[ogkm-hang] {_tag}end of dump\n")
                tf.flush()
                tf.seek(0)
                text = tf.read()
            time.sleep(0.3 * int(os.environ.get("LOCAL_RANK", "0") or 0))
            out.write(text)
            out.flush()
        except Exception:  # noqa: BLE001
            pass


def dumps() -> int:
    return _dumps


def _signal_loop() -> None:
    while True:
        sig = signal.sigwait({signal.SIGUSR1})
        if sig == signal.SIGUSR1:
            dump("SIGUSR1 (launcher timeout or operator request)")


def _watchdog_loop() -> None:
    global _deadline
    while True:
        time.sleep(1.0)
        d = _deadline
        if d is not None and time.monotonic() > d:
            _deadline = None
            dump(f"watchdog: '{_what}' still running after its deadline")


def install(tag: str = "") -> bool:
    """Start the dump thread (SIGUSR1) and the watchdog. Idempotent. Returns
    False when SIGUSR1 could not be routed to the dump thread (not the main
    thread, or no pthread_sigmask): the watchdog still works."""
    global _installed, _tag
    _tag = tag
    if _installed:
        return True
    _installed = True
    ok = False
    if threading.current_thread() is threading.main_thread() and hasattr(signal, "pthread_sigmask"):
        signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGUSR1})
        threading.Thread(target=_signal_loop, name="ogkm-hang-dump", daemon=True).start()
        ok = True
    threading.Thread(target=_watchdog_loop, name="ogkm-watchdog", daemon=True).start()
    return ok


def arm(seconds: float, what: str) -> None:
    """Dump once if ``what`` is still running ``seconds`` from now (``disarm`` ends it)."""
    global _deadline, _what
    _what = what
    _deadline = time.monotonic() + seconds


def disarm() -> None:
    global _deadline
    _deadline = None
