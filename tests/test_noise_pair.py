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
