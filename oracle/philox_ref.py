"""numpy Philox4x32-R and the noise streams of the kernels' Philox mode  —  TEST INFRASTRUCTURE ONLY.

Restates Salmon, Moraes, Dror & Shaw, "Parallel random numbers: as easy as 1, 2, 3"
(SC'11), Philox4x32 with R rounds (pertrenderer_amd/csrc/pr_common.h philox4x32<R>): the noise
streams use STREAM_ROUNDS = 7 (round 6; Crush-resistant per Salmon et al.), the round function is
pinned at R = 10 by Random123's known-answer vectors.  The counter layout the kernels use:
  rast:  counter (pixel, slot, sample // 4, 0x52415354), key = seed_r
  agg:   counter (pixel, slot, sample // 4, 0x41474752), key = seed_a
Each block gives 4 N(0,1) samples by Box-Muller (pr_common.h:gauss4).
Known-answer vectors from Random123's kat_vectors pin the generator itself.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
TAG_RAST, TAG_AGG = 0x52415354, 0x41474752
_MASK = np.uint64(0xFFFFFFFF)


STREAM_ROUNDS = 7  # pr_common.h PR_PHILOX_ROUNDS (include/pertrender.h PR_PHILOX_STREAM_ROUNDS)


def philox4x32_10(ctr, key):
    """Philox4x32-10 (Random123's known-answer vectors)."""
    return philox4x32(ctr, key, 10)


def philox4x32(ctr, key, rounds=STREAM_ROUNDS):
    """ctr: (...,4) uint32, key: (...,2) uint32 -> (...,4) uint32 after `rounds` rounds."""
    c = [np.asarray(ctr[..., i], np.uint32) for i in range(4)]
    k0 = np.asarray(key[..., 0], np.uint32).copy()
    k1 = np.asarray(key[..., 1], np.uint32).copy()
    with np.errstate(over="ignore"):
        for _ in range(rounds):
            p0 = M0 * c[0].astype(np.uint64)
            p1 = M1 * c[2].astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & _MASK).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & _MASK).astype(np.uint32)
            c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
            k0 = k0 + W0
            k1 = k1 + W1
    return np.stack(c, axis=-1)


def u01(r):
    """(r >> 8 | 1) * 2^-24, exactly as the kernels."""
    return (((np.asarray(r, np.uint32) >> np.uint32(8)) | np.uint32(1)).astype(np.float32)
            * np.float32(5.9604644775390625e-08))


def block(seed, pixel, slot, group, tag, rounds=STREAM_ROUNDS):
    pixel, slot, group = np.broadcast_arrays(np.asarray(pixel, np.uint32), np.asarray(slot, np.uint32),
                                             np.asarray(group, np.uint32))
    ctr = np.stack([pixel, slot, group, np.full(pixel.shape, tag, np.uint32)], axis=-1)
    key = np.array([seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF], np.uint32)
    return philox4x32(ctr, np.broadcast_to(key, ctr.shape[:-1] + (2,)), rounds)


def _bm4(w):
    """Box-Muller on one Philox block (...,4) -> 4 normals (float64 math; the kernels use
    the hardware log2/sqrt/sin/cos, so values agree to a few ulp)."""
    u = u01(w).astype(np.float64)
    r0 = np.sqrt(-2.0 * np.log(u[..., 0]))
    r1 = np.sqrt(-2.0 * np.log(u[..., 2]))
    return [r0 * np.cos(2 * np.pi * u[..., 1]), r0 * np.sin(2 * np.pi * u[..., 1]),
            r1 * np.cos(2 * np.pi * u[..., 3]), r1 * np.sin(2 * np.pi * u[..., 3])]


def _normals(seed, P, J, S, offset, tag):
    s = np.arange(offset, offset + S)
    pix = np.arange(P)[:, None]
    slot = np.arange(J)[None, :]
    out = np.empty((S, P, J), np.float64)
    for g in np.unique(s // 4):
        e = _bm4(block(seed, pix, slot, g, tag))                              # 4 x (P,J)
        for q in range(4):
            si = 4 * g + q - offset
            if 0 <= si < S:
                out[si] = e[q]
    return out


def rast_normals(seed, P, K, S, offset=0):
    """(S, P, K) Box-Muller normals of the rast stream (samples offset..offset+S-1)."""
    return _normals(seed, P, K, S, offset, TAG_RAST)


def agg_normals(seed, P, KP1, S, offset=0):
    """(S, P, K+1) Box-Muller normals of the agg stream."""
    return _normals(seed, P, KP1, S, offset, TAG_AGG)
