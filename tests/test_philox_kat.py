"""Known-answer tests of the Philox4x32 generator behind PR_NOISE_PHILOX.

The vectors are Random123's published kat_vectors for philox4x32_10 (Salmon et al., SC'11;
the three rows the Random123 distribution lists for R=10).  They pin the round function of
  * oracle/philox_ref.py (the numpy restatement, CPU test), and
  * the device generator itself, through the C-ABI entry pr_philox at 10 rounds (GPU test), which
    runs pr_common.h's philox4x32<R> / gauss4 / cauchy4 — the code the blend kernels draw with.
The streams run the same round function for PR_PHILOX_STREAM_ROUNDS = 7 rounds (round 6): the
device's 7-round blocks equal the restatement's bit for bit (test_device_noise_streams_...).
"""
import ctypes as C
import os

import numpy as np
import pytest
import torch

from oracle import philox_ref

# (counter, key) -> output, Random123 kat_vectors, "philox4x32 10" rows
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


def test_numpy_philox_matches_random123_kat():
    for ctr, key, out in KAT:
        got = philox_ref.philox4x32_10(np.array(ctr, np.uint32), np.array(key, np.uint32))
        assert [int(x) for x in got] == list(out)


def test_counter_layout_of_the_noise_streams():
    """block() puts (pixel, slot, sample group, tag) in the counter and the 64-bit seed in the key."""
    seed = 0x299f31d0_a4093822
    b = philox_ref.block(seed, 0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, rounds=10)
    assert [int(x) for x in b] == list(KAT[2][2])
    # the streams' rounds (7) by default, matching the header's constant
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                            "pertrender.h")).read()
    assert f"#define PR_PHILOX_STREAM_ROUNDS {philox_ref.STREAM_ROUNDS} " in hdr
    b7 = philox_ref.block(seed, 0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344)
    assert [int(x) for x in b7] != list(KAT[2][2])


def test_uniform_mapping_is_open_interval():
    u = philox_ref.u01(np.array([0, 0xffffffff, 0x100, 0x1ff], np.uint32))
    assert u[0] > 0 and u[1] < 1
    assert u[0] == np.float32(2.0 ** -24) and u[1] == np.float32(1 - 2.0 ** -24)


def _device_draw(ctr, keys, dev, rounds=philox_ref.STREAM_ROUNDS):
    from pertrenderer_amd import _native as nat
    lib = nat.load()
    n = ctr.shape[0]
    c = torch.from_numpy(np.ascontiguousarray(ctr, np.uint32).view(np.int32).copy()).to(dev)  # same bits
    k = torch.from_numpy(np.ascontiguousarray(keys, np.uint64).view(np.int64).copy()).to(dev)
    words = torch.empty((n, 4), dtype=torch.int32, device=dev)
    normals = torch.empty((n, 4), dtype=torch.float32, device=dev)
    cauchy = torch.empty((n, 4), dtype=torch.float32, device=dev)
    nat.check(lib.pr_philox(nat.ptr(c), nat.ptr(k), C.c_int64(n), nat.ptr(words), nat.ptr(normals),
                            nat.ptr(cauchy), C.c_int32(rounds), nat.stream_of(words)), "pr_philox")
    torch.cuda.synchronize()
    return (words.cpu().numpy().view(np.uint32), normals.cpu().numpy(), cauchy.cpu().numpy())


@pytest.mark.gpu
def test_device_philox_matches_random123_kat(device):
    ctr = np.array([c for c, _, _ in KAT], np.uint32)
    keys = np.array([k[0] | (k[1] << 32) for _, k, _ in KAT], np.uint64)
    words, _, _ = _device_draw(ctr, keys, device, rounds=10)
    np.testing.assert_array_equal(words, np.array([o for _, _, o in KAT], np.uint32))


@pytest.mark.gpu
def test_device_noise_streams_match_numpy_restatement(device):
    """Random counters of the rast / agg layout: words bit-exact, Box-Muller normals within a few
    ulp of the float64 restatement (the kernels use the hardware log2 / sqrt / sin / cos), Cauchy
    samples within 1e-5 relative away from the clamp."""
    rng = np.random.default_rng(0)
    n = 1 << 16
    ctr = rng.integers(0, 2 ** 32, (n, 4), dtype=np.uint64).astype(np.uint32)
    ctr[: n // 2, 3] = philox_ref.TAG_RAST
    ctr[n // 2:, 3] = philox_ref.TAG_AGG
    keys = rng.integers(0, 2 ** 63, n, dtype=np.uint64)
    words, normals, cauchy = _device_draw(ctr, keys, device)
    kw = np.stack([keys & np.uint64(0xFFFFFFFF), keys >> np.uint64(32)], -1).astype(np.uint32)
    ref_w = philox_ref.philox4x32(ctr, kw)  # the streams' rounds
    np.testing.assert_array_equal(words, ref_w)
    ref_n = np.stack(philox_ref._bm4(ref_w), -1)
    np.testing.assert_allclose(normals, ref_n, rtol=0, atol=2e-5 * np.maximum(1.0, np.abs(ref_n)).max())
    u = philox_ref.u01(ref_w).astype(np.float64)
    ref_c = np.clip(np.tan(np.pi * (u - 0.5)), -1e7, 1e7)
    mid = np.abs(ref_c) < 1e4  # the far tail is ill-conditioned in u (and clamped)
    np.testing.assert_allclose(cauchy[mid], ref_c[mid], rtol=1e-5, atol=1e-6)
    # moments of the normals (2^18 samples)
    assert abs(normals.mean()) < 0.01 and abs(normals.std() - 1.0) < 0.01
