"""The host staging extension (fedscale_amd/csrc/hoststage.c) on the CPU: it copies a small model's upload into the
pinned staging views exactly as the Python loop of ClientStaging._put_bulk_views does, and stops at the first entry
it does not take (wrong shape, dtype, byte order, layout, or not a plain ndarray) so that the Python loop converts
or raises as before; its build id is the tree's."""
import numpy as np
import pytest


def _dsts(shapes, dtypes):
    return [np.zeros(s, dtype=d) for s, d in zip(shapes, dtypes)]


def test_build_id_is_the_trees():
    from fedscale_amd import buildinfo, hoststage

    assert hoststage.load().build_id() == "FA_BUILD_ID=" + buildinfo.host_source_id()


def test_stage_copies_every_entry():
    from fedscale_amd import hoststage

    rng = np.random.default_rng(0)
    shapes, dtypes = [(10, 1, 5, 5), (10,), (), (0,), (3, 4)], [np.float32, np.float32, np.int64, np.float32, np.int64]
    vals = [np.asarray(rng.standard_normal(s) * 100).astype(d) for s, d in zip(shapes, dtypes)]
    d = _dsts(shapes, dtypes)
    assert hoststage.stage(vals, d) == -1
    for a, b in zip(vals, d):
        np.testing.assert_array_equal(a, b)
        assert a.dtype == b.dtype


@pytest.mark.parametrize("bad", ["shape", "dtype", "swapped", "strided", "list", "subclass", "f64"])
def test_stage_stops_at_the_first_entry_it_does_not_take(bad):
    from fedscale_amd import hoststage

    shapes, dtypes = [(4, 6), (6,), (2, 3)], [np.float32, np.float32, np.float32]
    vals = [np.full(s, i + 1, dtype=np.float32) for i, s in enumerate(shapes)]
    v1 = {"shape": np.ones((6, 1), np.float32), "dtype": np.ones(6, np.int32), "f64": np.ones(6, np.float64),
          "swapped": np.ones(6, np.dtype(">f4")), "strided": np.ones(12, np.float32)[::2],
          "list": [1.0] * 6, "subclass": np.ones(6, np.float32).view(np.matrix)}[bad]
    vals[1] = v1
    d = _dsts(shapes, dtypes)
    assert hoststage.stage(vals, d) == 1
    np.testing.assert_array_equal(d[0], vals[0])  # the entries before it were copied
    assert not d[1].any() and not d[2].any()  # nothing from it on


def test_stage_rejects_mismatched_lengths():
    from fedscale_amd import hoststage

    with pytest.raises(ValueError):
        hoststage.stage([np.ones(2, np.float32)], [])


def test_copies_at_every_offset_and_length():
    """Destinations at every 4-byte offset of a 16-byte line, lengths around the copy's block sizes: the same bytes,
    nothing written outside the destination."""
    from fedscale_amd import hoststage

    rng = np.random.default_rng(1)
    big = np.zeros(70_000, np.float32)
    for off in range(4):
        for n in (1, 255, 256, 257, 4099, 12_345):
            src = rng.standard_normal(n).astype(np.float32)
            big[:] = 0
            dst = big[off:off + n]
            assert hoststage.stage([src], [dst]) == -1
            np.testing.assert_array_equal(dst, src)
            assert not big[:off].any() and not big[off + n:].any()
