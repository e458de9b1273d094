"""Property tests (hypothesis) of the bucket layout: for any state_dict shape list and any world size,
the shards tile the fp32 vector exactly, are balanced (within 64 floats) and 64-aligned, and pack -> gather -> unpack is
the identity (the host half of the sharded path; CPU only)."""
import numpy as np
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from fedscale_amd.bucket import ALIGN, BucketLayout

shape = st.lists(st.integers(0, 9), min_size=0, max_size=3).map(tuple)
entry = st.tuples(shape, st.sampled_from([torch.float32, torch.float32, torch.int64]))


@settings(max_examples=60, deadline=None)
@given(st.lists(entry, min_size=1, max_size=8), st.integers(1, 9), st.integers(0, 2**31 - 1))
def test_shards_tile_and_roundtrip(entries, world, seed):
    names = [f"e{i}" for i in range(len(entries))]
    shapes = [e[0] for e in entries]
    dtypes = [e[1] for e in entries]
    full = BucketLayout(names, shapes, dtypes)
    rng = np.random.default_rng(seed)
    vals = [rng.normal(size=s).astype(np.float32) if d == torch.float32
            else np.asarray(rng.integers(-5, 5, size=s), dtype=np.int64) for s, d in zip(shapes, dtypes)]
    parts = []
    side = None
    ld0 = BucketLayout(names, shapes, dtypes, 0, world).ld
    for r in range(world):
        lay = BucketLayout(names, shapes, dtypes, r, world)
        assert lay.ld == ld0 and lay.ld % ALIGN == 0 and lay.P <= lay.ld
        f = np.zeros(lay.ld, np.float32)
        i = np.zeros(lay.ldq, np.int64)
        lay.pack_host(vals, f, i, workers=2)
        parts.append(f)
        side = i if side is None else side
        np.testing.assert_array_equal(side, i)  # the side table is replicated
    assert sum(BucketLayout(names, shapes, dtypes, r, world).P for r in range(world)) == full.P_full
    flat = BucketLayout(names, shapes, dtypes, 0, world).unshard(np.concatenate(parts))  # the all-gather's rows
    out = full.unpack(torch.from_numpy(np.ascontiguousarray(flat)), torch.from_numpy(side))
    for o, v in zip(out, vals):
        np.testing.assert_array_equal(o.numpy(), v)


@settings(max_examples=500, deadline=None)
@given(st.integers(0, 10**9), st.integers(1, 16))
def test_shard_bounds_balanced_and_aligned(P, world):
    """Parameter slices (bucket.shard_bounds): they tile [0, P) in rank order, every boundary is a multiple of 64,
    every slice holds P/world floats within 64 (when P >= 64*world), and the common row stride ld holds each."""
    from fedscale_amd.bucket import shard_bounds, shard_ld

    b = shard_bounds(P, world)
    assert b[0] == 0 and b[-1] == P and all(b[r] <= b[r + 1] for r in range(world))
    assert all(x % ALIGN == 0 or x == P for x in b[:-1])  # (slices past the end are empty)
    sizes = [b[r + 1] - b[r] for r in range(world)]
    if P >= 64 * world:
        assert max(abs(s_ - P / world) for s_ in sizes) <= 64
    ld = shard_ld(P, world)
    assert ld % ALIGN == 0 and max(sizes) <= ld < max(sizes) + ALIGN + (ALIGN if max(sizes) == 0 else 0)


def test_eight_way_split_of_config5():
    """BASELINE config 5's 100 M parameters over 8 GPUs: 64-aligned slices within 64 floats of 12.5 M."""
    from fedscale_amd.bucket import shard_bounds, shard_ld

    b = shard_bounds(100_000_000, 8)
    sizes = [b[r + 1] - b[r] for r in range(8)]
    assert sizes == [12_499_968, 12_500_032] * 4 and shard_ld(100_000_000, 8) == 12_500_032
    assert all(x % 64 == 0 for x in b[:-1]) and max(sizes) - min(sizes) == 64


@settings(max_examples=200, deadline=None)
@given(st.integers(1, 5000), st.integers(1, 16))
def test_client_blocks_partition_arrivals(K, world):
    """Client mode (state.py): the ranks' arrival blocks are contiguous, in rank order, cover 0..K-1
    exactly once, differ in size by at most one, and owner() names the block holding each arrival."""
    from fedscale_amd.state import ShardGroup

    g = ShardGroup(0, world, mode="clients")
    blocks = [g.client_block(K, r) for r in range(world)]
    assert blocks[0][0] == 0 and blocks[-1][1] == K
    assert all(blocks[r][1] == blocks[r + 1][0] for r in range(world - 1))
    sizes = [b - a for a, b in blocks]
    assert max(sizes) - min(sizes) <= 1
    ks = np.unique(np.linspace(0, K - 1, num=min(K, 64)).astype(int))
    for k in ks:
        a, b = blocks[g.owner(int(k), K)]
        assert a <= k < b


def test_piece_segments_cover_every_slice_exactly():
    """RegisteredUpload's segments (fedscale_amd/bucket.py PieceSegments, round-4 N-GPU ingress): the whole-model
    segments tile [0, P) in order; each large entry is one segment; every part's pieces tile its slice [p0, p1)
    exactly, each piece inside one segment; empty entries take no piece."""
    import numpy as np
    import torch

    from fedscale_amd.bucket import BucketLayout, PieceSegments, shard_bounds

    rng = np.random.default_rng(3)
    for trial in range(20):
        T = int(rng.integers(1, 30))
        shapes = [(int(rng.choice([0, 1, 7, 300, 70_000, 300_000])),) for _ in range(T)]
        dtypes = [torch.float32 if rng.random() < 0.9 else torch.int64 for _ in range(T)]
        L = BucketLayout([f"t{i}" for i in range(T)], shapes, dtypes)
        segs = PieceSegments(L, min_bytes=4 * 70_000)
        pos = 0
        for off, n, k in segs.segs:
            assert off == pos and n > 0
            pos += n
        assert pos == L.P_full
        large = [e for e in L.f_entries if e.numel >= 70_000]
        assert [segs.segs[i][1] for i in range(len(segs.segs)) if segs.segs[i][2] >= 0] == [e.numel for e in large]
        assert len(segs.large_pieces) + len(segs.small_pieces) == sum(1 for e in L.f_entries if e.numel)
        for N in (1, 2, 3, 8):
            bnd = shard_bounds(L.P_full, N)  # BucketLayout's slices
            for r in range(N):
                p0, p1 = bnd[r], bnd[r + 1]
                dst, nb, kind, soff = segs.part_plan(p0, p1)
                got = sum(int(b) for b in nb)
                assert got == 4 * (p1 - p0)
                cur = 0
                for d, b in zip(dst.tolist(), nb.tolist()):
                    assert d == cur and b > 0
                    cur += b
