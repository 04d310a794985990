"""Several batches in flight on one GPU: N casr handles bound to one packed weight blob, each
on a HIP stream of its own; batch i is enqueued on handle i mod N.

A batch's chain (features -> encoder -> decode) is serial: its decode cannot
start before its encoder ends, and most of its kernels leave parts of the chip idle (the
recurrence is latency-bound, the decode GEMMs and the attention are bound by per-CU intake, the
small launches of the decode steps leave gaps).  With two batches in flight the hardware
interleaves one batch's work with the other's (measured at B = 256 greedy: 6.54 -> 6.16-6.21 ms
per batch, tools/probes/two_stream_probe.py).  Nothing is shared between the
handles but the read-only weight blob, so each batch's results are bitwise those of a decode on
one handle alone (tests/test_gpu_pipeline.py).

The reference decodes one batch at a time on the host (model.py:503-987); this is the serving
loop around the same per-batch call, not a change of what a batch computes.
"""
import torch

from .engine import Engine


class StreamPipeline:
    """`n` Engines on `n` streams sharing `packed` (a device blob: the bytes every rank receives
    from broadcast_packed, or casr.lib.pack_weights' output moved to the device)."""

    def __init__(self, cfg, packed, n=2, device=None):
        if n < 1:
            raise ValueError("a pipeline needs at least one handle")
        self.engines = [Engine(cfg, packed=packed, device=device) for _ in range(n)]
        dev = self.engines[0].device
        # handle 0 keeps the caller's current stream (a one-handle pipeline is the plain serial
        # loop); the others get streams of their own
        self.streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(n - 1)]
        self.n = n
        self.cfg = cfg
        self._next = 0

    def limited(self, n):
        """A view that submits round-robin over the first n handles only (same handles, same
        streams): one pipeline object serves workloads that want different depths."""
        return _Limited(self, n)

    def submit(self, fn, n=None):
        """Enqueue fn(engine) for the next batch on its handle's stream and return what fn
        returns (device tensors produced on that stream).  The inputs fn reads must be complete
        before the call (staged and synchronised, as bench.py does, or guarded by an event the
        caller waits on inside fn): no stream here waits on another, which is what lets batch i
        run beside batch i - 1."""
        j = self._next % (n or self.n)
        self._next += 1
        s = self.streams[j]
        with torch.cuda.stream(s):
            return fn(self.engines[j])

    def reset(self):
        """Next batch on handle 0 again (after a synchronize)."""
        self._next = 0

    def set_precision(self, p):
        for e in self.engines:
            e.set_precision(p)

    def set_option(self, name, value):
        for e in self.engines:
            e.set_option(name, value)

    def set_graphs(self, mode):
        for e in self.engines:
            e.set_graphs(mode)

    def precision(self):
        return self.engines[0].precision()

    def device_flags(self):
        """Guard bits of every handle since the previous read (OR; synchronises each stream)."""
        f = 0
        for e, s in zip(self.engines, self.streams):
            with torch.cuda.stream(s):
                f |= e.device_flags()
        return f

    def profile(self, classes):
        for e in self.engines:
            e.profile(classes)

    def profile_read(self):
        """{class: (launches, total_ms)} summed over the handles (each launch timed on its own
        stream, so overlapped launches each count their own span)."""
        out = {}
        for e in self.engines:
            for c, (n, ms) in e.profile_read().items():
                a, b = out.get(c, (0, 0.0))
                out[c] = (a + n, b + ms)
        return out

    def close(self):
        for e in self.engines:
            e.close()


class _Limited:
    def __init__(self, pipe, n):
        self.pipe, self.n = pipe, min(n, pipe.n)
        self.cfg = pipe.cfg
        self.engines = pipe.engines[:self.n]

    def submit(self, fn):
        return self.pipe.submit(fn, self.n)

    def device_flags(self):
        f = 0
        for e, s in zip(self.engines, self.pipe.streams):
            with torch.cuda.stream(s):
                f |= e.device_flags()
        return f
