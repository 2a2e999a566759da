"""Per-kernel HIP-event timing for bench.py's roofline leg.

When a :class:`KernelTimer` is active (``with KernelTimer() as t``), every native
launch site brackets its kernel with two events recorded on the SAME stream the
kernel is enqueued on (torch's current stream of the tensors' device), so the
elapsed time is the kernel's own duration on that stream.

In an eager (uncaptured) pass the GPU is usually AHEAD of the host: it would reach the
start event before the host has submitted the launch, and the interval would include
host time (Python, argument packing).  ``lead_cycles`` enqueues a device-side spin
(``torch.cuda._sleep``) before the start event, long enough for the host to submit the
launch behind it, so start event -> kernels -> stop event run back to back on the GPU.
"""
import collections

import torch

_ACTIVE = None


def active():
    return _ACTIVE


class KernelTimer:
    """external=True creates events that become record nodes when the launches are
    captured into a HIP graph; after a replay they time that replay's kernels."""

    def __init__(self, external=False, lead_cycles=0, warm_bytes=0):
        self._open = {}
        self.events = collections.defaultdict(list)
        self.external = external
        self.lead_cycles = lead_cycles
        # after the (single-wave) spin the chip is idle and its clocks drop; a short full-chip
        # elementwise pass right before the start event brings them back before the timed launch
        self._warm = (torch.empty(warm_bytes // 4, dtype=torch.float32, device="cuda").fill_(1.0)
                      if warm_bytes else None)

    def __enter__(self):
        global _ACTIVE
        self._prev, _ACTIVE = _ACTIVE, self
        return self

    def __exit__(self, *exc):
        global _ACTIVE
        _ACTIVE = self._prev
        return False

    def start(self, name):
        if self.lead_cycles and hasattr(torch.cuda, "_sleep"):
            torch.cuda._sleep(self.lead_cycles)
        if self._warm is not None:
            self._warm.mul_(1.0)
        ev = torch.cuda.Event(enable_timing=True, external=self.external)
        ev.record(torch.cuda.current_stream())
        self._open[name] = ev

    def stop(self, name):
        ev = torch.cuda.Event(enable_timing=True, external=self.external)
        ev.record(torch.cuda.current_stream())
        self.events[name].append((self._open.pop(name), ev))

    def reset(self):
        self.events.clear()

    def summary(self, stat="mean"):
        """{name: (launches, ms)} with ms the mean, median or minimum over launches — call after
        torch.cuda.synchronize()."""
        out = {}
        for name, pairs in self.events.items():
            ms = sorted(a.elapsed_time(b) for a, b in pairs)
            if not ms:
                continue
            if stat == "median":
                m = len(ms) // 2
                v = ms[m] if len(ms) % 2 else 0.5 * (ms[m - 1] + ms[m])
            elif stat == "min":
                v = ms[0]
            else:
                v = sum(ms) / len(ms)
            out[name] = (len(ms), v)
        return out
