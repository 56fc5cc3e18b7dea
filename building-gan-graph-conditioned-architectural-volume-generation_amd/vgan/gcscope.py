"""The host loops that feed the GPU, out of the cyclic GC's way.

A fresh-batch training step (``Trainer._train_batch`` -> ``step_fresh``)
creates thousands of short-lived Python objects (ctypes descriptors, tensor
views, batch objects), so the interpreter runs generation-0 collections
every few launches and a full collection every ~10 of those; a full
collection traverses every tracked object in the process.  With a second
trainer, a pool of resident batches and their recorded graphs alive beside
it, the fresh leg took 10.6-11.4 ms per step against 8.3-8.4 ms with them
released or frozen (profiles/r04_gc_freeze_ab.txt).  ``gc_frozen`` moves
everything alive when the loop starts into the permanent generation
(``gc.freeze``: O(1), nothing is collected or copied), so the loop's
collections only traverse what the loop itself allocates; the objects are
handed back on exit (``gc.unfreeze``).  Nested uses freeze once.
"""
from __future__ import annotations

import contextlib
import gc
import threading

_lock = threading.Lock()
_depth = 0


@contextlib.contextmanager
def gc_frozen():
    global _depth
    with _lock:
        if _depth == 0:
            gc.freeze()
        _depth += 1
    try:
        yield
    finally:
        with _lock:
            _depth -= 1
            if _depth == 0:
                gc.unfreeze()
