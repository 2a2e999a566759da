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

Besides the call-level pair, the timer arms the library's own kernel timer
(``pr_ktimer_arm``): the native call then records a second pair on its launch stream
right around its dominant kernel (blend_fwd_kernel, blend_bwd_kernel, rast_fwd_kernel,
rast_bwd_kernel), so ``kernel_summary`` reports that kernel's duration alone, named as
rocprofv3 names it -- the basis of bench.py's roofline.
"""
import collections
import ctypes

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
        self.kslots = collections.defaultdict(list)  # call name -> [native timer slot per launch]
        self._nslot = 0
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
        if not self.external and self._nslot < 256:
            from . import _native as nat
            if nat.load().pr_ktimer_arm(self._nslot) == 0:
                self.kslots[name].append(self._nslot)
                self._nslot += 1

    def stop(self, name):
        ev = torch.cuda.Event(enable_timing=True, external=self.external)
        ev.record(torch.cuda.current_stream())
        self.events[name].append((self._open.pop(name), ev))
        if not self.external:
            from . import _native as nat
            nat.load().pr_ktimer_arm(-1)  # a call that launched no timed kernel leaves nothing armed

    def reset(self):
        self.events.clear()
        self.kslots.clear()
        self._nslot = 0

    def kernel_summary(self, stat="mean"):
        """{call name: (kernel name, launches, ms)} of the dominant kernel of each native call,
        from the library's own event pair around that kernel -- after torch.cuda.synchronize()."""
        from . import _native as nat
        lib = nat.load()
        out = {}
        for name, slots in self.kslots.items():
            ms, kname = [], None
            for s in slots:
                v, buf = ctypes.c_float(), ctypes.create_string_buffer(64)
                if lib.pr_ktimer_read(s, ctypes.byref(v), buf, 64) == 0:
                    ms.append(v.value)
                    kname = buf.value.decode()
            if ms:
                out[name] = (kname, len(ms), _stat(sorted(ms), stat))
        return out

    def summary(self, stat="mean"):
        """{name: (launches, ms)} with ms the mean, median or minimum over launches — call after
        torch.cuda.synchronize()."""
        out = {}
        for name, pairs in self.events.items():
            ms = sorted(a.elapsed_time(b) for a, b in pairs)
            if ms:
                out[name] = (len(ms), _stat(ms, stat))
        return out


def _stat(ms, stat):
    """mean / median / min of a sorted list."""
    if stat == "median":
        m = len(ms) // 2
        return ms[m] if len(ms) % 2 else 0.5 * (ms[m - 1] + ms[m])
    if stat == "min":
        return ms[0]
    return sum(ms) / len(ms)
