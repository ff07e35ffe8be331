"""Decode split planner (ops.decode_split_plan): every plan covers the context
with 64-key multiples, respects a captured grid's split cap, and picks the
round-filling split counts measured on MI355X (profiles/decode_nsplit.txt)."""
import math

import pytest

from llmd_amd import ops


@pytest.mark.parametrize("batch", [1, 3, 8, 24, 48, 64, 96, 110, 160, 256])
@pytest.mark.parametrize("ctx", [1, 63, 64, 65, 700, 5125, 7416, 32768])
@pytest.mark.parametrize("G", [1, 4, 8, 16, 20])
def test_plan_covers_context(batch, ctx, G):
    split, n = ops.decode_split_plan(ctx, batch, 8, G)
    assert split % 64 == 0 and split >= 64 and n >= 1
    assert split * n >= ctx and split * (n - 1) < max(ctx, 1)  # no empty split
    capped = ops.decode_split_plan(ctx, batch, 8, G, max_splits=2)
    assert capped[1] <= 2 and capped[0] * capped[1] >= ctx


def test_plan_fills_workgroup_rounds():
    # 48 x 8 heads = 384 workgroups: 4 splits make 3 full rounds of 512 (measured 293 -> 264 us)
    assert ops.decode_split_plan(7416, 48, 8, 8)[1] == 4
    # 64 x 8 = 512 workgroups: exactly one round with one split
    assert ops.decode_split_plan(5125, 64, 8, 8)[1] == 1
    # batch 1 long context: many splits to spread one sequence over the chip
    assert ops.decode_split_plan(32768, 1, 8, 8)[1] >= 16
    # beyond two rounds the tail shrinks: 160 x 8 stays at one split
    assert ops.decode_split_plan(3000, 160, 8, 8)[1] == 1


def test_graph_replay_split_within_grid():
    """The runner re-sizes a captured grid's splits to the step: split x cap >= context."""
    for cap in (1, 2, 4, 16):
        for ctx in (100, 2000, 9000):
            split, n = ops.decode_split_plan(ctx, 20, 8, 8, max_splits=cap)
            assert n <= cap and split * cap >= ctx and split == math.ceil(split / 64) * 64
