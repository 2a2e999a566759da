"""Noise sources for the perturbed operators.

Two sources, selected globally with :func:`set_noise_source` or per call with a
:class:`Noise` object:

``"philox"`` (default, production)
    In-kernel Philox4x32-10.  Each operator call draws one 62-bit key from
    torch's default CPU generator (so ``torch.manual_seed`` makes runs
    reproducible, and the rast draw precedes the agg draw exactly as in the
    reference: smoothrast.py:21 then smoothagg.py:21).  Noise is a pure function
    of (key, pixel, slot, sample): nothing of size S x P x K is stored, the
    backward regenerates it, and disjoint sample ranges (``sample_offset``)
    give independent shards for multi-GPU sample parallelism.

``"torch"`` (reference parity)
    The N(0,1) tensors are drawn on the CPU with ``torch.randn`` in the shapes
    and order the reference draws them ((Sr,N,H,W,K) then (Sa,N,H,W,K+1),
    including ``fixed_noise``'s ``torch.manual_seed(1)``), copied to the device
    and read by the kernels.  With the same seed this reproduces the
    reference's CPU outputs.
"""
from dataclasses import dataclass
from typing import Optional

import torch

from . import _native as nat

_SOURCE = "philox"
SOURCES = ("philox", "torch")


def set_noise_source(name):
    global _SOURCE
    if name not in SOURCES:
        raise ValueError(f"noise source must be one of {SOURCES}, got {name!r}")
    _SOURCE = name


def get_noise_source():
    return _SOURCE


def draw_key(generator=None):
    """One 62-bit Philox key from torch's (CPU) generator."""
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64, generator=generator).item())


@dataclass
class Noise:
    """Noise of one operator call (kept by autograd for the backward)."""
    mode: int
    seed_r: int = 0
    seed_a: int = 0
    noise_r: Optional[torch.Tensor] = None
    noise_a: Optional[torch.Tensor] = None
    offset_r: int = 0
    offset_a: int = 0
    seeds: Optional[torch.Tensor] = None  # device int64[1] key base (graph mode)

    @staticmethod
    def philox(seed_r=0, seed_a=0, offset_r=0, offset_a=0, seeds=None):
        return Noise(nat.PR_NOISE_PHILOX, int(seed_r), int(seed_a), None, None, int(offset_r),
                     int(offset_a), seeds)

    @staticmethod
    def injected(noise_r=None, noise_a=None):
        return Noise(nat.PR_NOISE_INJECTED, 0, 0, noise_r, noise_a, 0, 0)

    def to(self, device):
        if self.noise_r is None and self.noise_a is None:  # Philox: nothing on the host to move
            return self
        mv =(lambda t: None if t is None else t.to(device=device, dtype=torch.float32).contiguous())
        return Noise(self.mode, self.seed_r, self.seed_a, mv(self.noise_r), mv(self.noise_a),
                     self.offset_r, self.offset_a, self.seeds)


class DeviceSeed:
    """Graph-capturable Philox keys.

    A device-resident 64-bit base is advanced in place by ``advance()``; every operator call in
    between gets a distinct stream id, and the kernels key Philox with mix64(base ^ id).  Inside a
    captured step the ids are baked into the graph while the base changes per replay, so every
    replay draws fresh noise without any host work.

    The advance is deferred (round 5): ``advance()`` only counts it, and the next native face pass
    (``MeshRasterizer`` -> pr_project_rast_fwd, PRProjectArgs.seed_advance) applies it in its first
    thread, so a pose-optimisation step spends no launch of its own on it; any draw from this seed
    before such a pass (``stream_id``) flushes the pending advances with pr_seed_advance first, so
    the keys every operator sees are those of the eager update."""

    def __init__(self, device, seed=None):
        self.tensor = torch.tensor([draw_key() if seed is None else int(seed)], dtype=torch.int64,
                                   device=device)
        self._next = 1
        self._pending = 0

    def stream_id(self):
        self.flush()
        i = self._next
        self._next += 1
        return i

    def advance(self):
        self._pending += 1
        self._next = 1

    def flush(self):
        """Apply the pending advances now (pr_seed_advance on the current stream)."""
        while self._pending:
            nat.call("pr_seed_advance", "pr_seed_advance", self.tensor, nat.ptr(self.tensor), 1)
            self._pending -= 1

    def take_pending(self, device):
        """(tensor, n) of the pending advances for a native face pass on `device` to apply (n = 0:
        none); the caller owns them from here (give_back on failure)."""
        if not self._pending or self.tensor.device != device:
            return None, 0
        n, self._pending = self._pending, 0
        return self.tensor, n

    def give_back(self, n):
        self._pending += n


def take_pending_advance(device):
    """The active DeviceSeed's deferred advances for a face pass on `device`: (tensor, n)."""
    if _DEVICE_SEED is None:
        return None, 0
    return _DEVICE_SEED.take_pending(device)


def give_back_advance(n):
    if n and _DEVICE_SEED is not None:
        _DEVICE_SEED.give_back(n)


_DEVICE_SEED = None
_SHARD = 0  # this process's Monte-Carlo sample shard index (set_sample_shard)
_OFFSET = None  # explicit global (rast, agg) sample offsets (set_sample_offset), override the shard index


def set_sample_shard(index):
    """Sample-parallel rendering (BASELINE north star): every Philox draw of an
    operator with S samples takes the global sample indices [index*S, (index+1)*S) of one
    estimator, so ranks sharing keys (same seed / DeviceSeed base) draw disjoint sample shards
    of the same frame, and averaging their gradients (parallel.average_gradients) is the
    (world*S)-sample estimator.  Index 0 (default) is the single-process behaviour."""
    global _SHARD
    _SHARD = int(index)


def sample_shard():
    return _SHARD


def set_sample_offset(offset_r, offset_a=None):
    """Draw the rast (agg) operators' samples from global index offset_r (offset_a) on; None
    restores the shard index's offsets.  Uneven sample shards (parallel.sample_shard) of one
    estimator use this."""
    global _OFFSET
    _OFFSET = None if offset_r is None else (int(offset_r), int(offset_r if offset_a is None else offset_a))


def _offset(S, which):
    return _OFFSET[which] if _OFFSET is not None else _SHARD * S


def use_device_seed(ds):
    """Route Philox draws through a :class:`DeviceSeed` (None restores host draws)."""
    global _DEVICE_SEED
    _DEVICE_SEED = ds


def _torch_draw(kind, shape):
    """The reference's draws on the CPU generator: torch.normal(0, 1) (smoothrast.py:21,
    smoothagg.py:21), Cauchy(0, 1) samples clamped to +-1e7 (smoothrast.py:23-24,
    smoothagg.py:26-27) or Uniform(-1/2, 1/2) samples (smoothagg.py:28-30)."""
    if kind == "gaussian":
        return torch.randn(shape)
    if kind == "uniform":  # smoothagg.py:28-30
        m = torch.distributions.uniform.Uniform(torch.tensor([-0.5]), torch.tensor([0.5]))
        return m.sample(shape).squeeze(-1)
    m = torch.distributions.cauchy.Cauchy(torch.tensor([0.0]), torch.tensor([1.0]))
    return torch.clamp(m.sample(shape).squeeze(-1), min=-1e7, max=1e7)


def draw_rast(shape, Sr, device, kind="gaussian"):
    """Noise for one perturbed-Heaviside call over fragments of `shape` (N,H,W,K)."""
    if _SOURCE == "torch":
        return Noise.injected(noise_r=_torch_draw(kind, (Sr,) + tuple(shape)).to(device))
    if _DEVICE_SEED is not None:
        return Noise.philox(seed_r=_DEVICE_SEED.stream_id(), seeds=_DEVICE_SEED.tensor, offset_r=_offset(Sr, 0))
    return Noise.philox(seed_r=draw_key(), offset_r=_offset(Sr, 0))


def draw_agg(shape, Sa, device, fixed_noise=False, kind="gaussian"):
    """Noise for one perturbed-argmax call over logits of `shape` (N,H,W,K+1).
    fixed_noise reseeds the global generator with 1 first, as smoothagg.py:18-19
    (and then ignores any device seed: the noise must be the same every call)."""
    if fixed_noise:
        torch.manual_seed(1)
    if _SOURCE == "torch":
        return Noise.injected(noise_a=_torch_draw(kind, (Sa,) + tuple(shape)).to(device))
    if _DEVICE_SEED is not None and not fixed_noise:
        return Noise.philox(seed_a=_DEVICE_SEED.stream_id(), seeds=_DEVICE_SEED.tensor, offset_a=_offset(Sa, 1))
    return Noise.philox(seed_a=draw_key(), offset_a=_offset(Sa, 1))


def draw_pair(shape, Sr, Sa, device, fixed_noise=False, rast_kind="gaussian", agg_kind="gaussian"):
    """(rast draw, agg draw) of one fused blend call, as draw_rast then draw_agg.  With host-keyed
    Philox and no fixed_noise both keys come from ONE randint of two values: the CPU generator
    yields the same two 64-bit draws in the same order as two one-value calls (checked in
    tests/test_noise_pair.py), for half the host time.  None in the other modes (the caller draws
    one by one)."""
    if _SOURCE != "philox" or _DEVICE_SEED is not None or fixed_noise:
        return None
    k = torch.randint(0, 2 ** 62, (2,), dtype=torch.int64).tolist()
    return (Noise.philox(seed_r=k[0], offset_r=_offset(Sr, 0)), Noise.philox(seed_a=k[1], offset_a=_offset(Sa, 1)))

