"""noise.draw_pair (both Philox keys of a fused blend call from one randint) draws exactly the keys
draw_rast then draw_agg would, in every mode where it applies, and declines the others."""
import torch

from pertrenderer_amd import noise as nm


def test_pair_equals_sequential_draws():
    for seed in (0, 5, 123):
        torch.manual_seed(seed)
        r, a = nm.draw_rast((1, 4, 4, 3), 8, None), nm.draw_agg((1, 4, 4, 4), 8, None)
        torch.manual_seed(seed)
        pr, pa_ = nm.draw_pair((1, 4, 4, 3), 8, 8, None)
        assert (pr.seed_r, pa_.seed_a, pr.offset_r, pa_.offset_a) == (r.seed_r, a.seed_a, r.offset_r, a.offset_a)


def test_pair_keeps_generator_state():
    torch.manual_seed(9)
    nm.draw_rast((1, 2, 2, 2), 4, None)
    nm.draw_agg((1, 2, 2, 3), 4, None)
    after_seq = torch.randint(0, 2 ** 62, (1,)).item()
    torch.manual_seed(9)
    nm.draw_pair((1, 2, 2, 2), 4, 4, None)
    assert torch.randint(0, 2 ** 62, (1,)).item() == after_seq


def test_pair_declines_other_modes():
    assert nm.draw_pair((1, 2, 2, 2), 4, 4, None, fixed_noise=True) is None
    nm.set_noise_source("torch")
    try:
        assert nm.draw_pair((1, 2, 2, 2), 4, 4, None) is None
    finally:
        nm.set_noise_source("philox")


def test_pair_shard_offsets():
    nm.set_sample_shard(2)
    try:
        r, a = nm.draw_pair((1, 2, 2, 2), 4, 6, None)
        assert (r.offset_r, a.offset_a) == (8, 12)
    finally:
        nm.set_sample_shard(0)


def test_fixed_noise_two_call_sequence_follows_the_reference_reseed_order():
    """fixed_noise=True: randomArgmax.forward calls torch.manual_seed(1) before ITS draw
    (smoothagg.py:18-19), after randomHeaviside.forward drew the rast noise from the caller's
    generator state (smoothrast.py:21).  So call 1's rast noise differs from call 2's, and every later
    call repeats call 2 -- the reference's semantics, not a first-use defect.  Pinned against the
    reference's own draw order (torch.normal(mean=zeros, std=1.), as smoothrast.py:21 / smoothagg.py:21)
    in the parity noise source, and for the Philox keys in the default one."""
    shape_r, shape_a, Sr, Sa = (1, 3, 4, 5), (1, 3, 4, 6), 4, 3
    nm.set_noise_source("torch")
    try:
        torch.manual_seed(123)
        got = [(nm.draw_rast(shape_r, Sr, "cpu").noise_r, nm.draw_agg(shape_a, Sa, "cpu", fixed_noise=True).noise_a)
               for _ in range(3)]
    finally:
        nm.set_noise_source("philox")
    torch.manual_seed(123)
    exp = []
    for _ in range(3):
        r = torch.normal(mean=torch.zeros((Sr,) + shape_r), std=1.)  # smoothrast.py:21
        torch.manual_seed(1)  # smoothagg.py:18-19
        a = torch.normal(mean=torch.zeros((Sa,) + shape_a), std=1.)  # smoothagg.py:21
        exp.append((r, a))
    for (gr, ga), (er, ea) in zip(got, exp):
        assert torch.equal(gr, er) and torch.equal(ga, ea)
    assert not torch.equal(got[0][0], got[1][0])  # call 1's rast noise: the caller's state
    assert torch.equal(got[1][0], got[2][0])  # later calls repeat call 2
    assert torch.equal(got[0][1], got[1][1]) and torch.equal(got[1][1], got[2][1])
    # Philox keys: the same order (the rast key from the caller's state, the agg key after the reseed)
    torch.manual_seed(123)
    keys = [(nm.draw_rast(shape_r, Sr, None).seed_r, nm.draw_agg(shape_a, Sa, None, fixed_noise=True).seed_a)
            for _ in range(3)]
    assert keys[0][0] != keys[1][0] and keys[1] == keys[2] and keys[0][1] == keys[1][1]
