"""Small rounds read the staged updates out of the pinned mirror and write the new model into its egress
snapshot (fa_reduce_mirror).  Same arithmetic and order as fa_reduce, so every result
is bit-exact against the oracle; the tests also pin down which buffers the kernels actually touched and that
a snapshot a reader holds never changes under it."""
import numpy as np
import pytest
import torch

from oracle.cpu_reference import fedavg_close, fedavg_flat, fedavg_step, fedbuff_flat
from tests.golden_io import StateDictModule, assert_state_equal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,P", [(10, 24492), (3, 5), (64, 1001), (1, 4096)])
@pytest.mark.parametrize("x_host", [True, False], ids=["x_pinned", "x_device"])
@pytest.mark.parametrize("mirror_host", [True, False], ids=["mirror_pinned", "mirror_device"])
def test_reduce_mirror_bit_exact(gpu_device, K, P, x_host, mirror_host):
    from fedscale_amd import kernels as kx

    ld = (P + 63) // 64 * 64
    rng = np.random.default_rng(K * 7 + P)
    xh = torch.from_numpy(rng.standard_normal((K, ld), dtype=np.float32))
    xh[:, P:] = 0
    x = xh.pin_memory() if x_host else xh.to(gpu_device)
    out = torch.full((ld,), np.nan, device=gpu_device)
    mirror = torch.full((ld,), np.nan).pin_memory() if mirror_host else torch.full((ld,), np.nan, device=gpu_device)
    a = torch.from_numpy(rng.uniform(0.2, 1.0, K).astype(np.float32)).to(gpu_device)
    kx.reduce_mirror(x, K, P, out, mirror, denom=float(np.float32(K)))
    torch.cuda.synchronize()
    want = fedavg_flat(xh[:K, :P].numpy())
    assert np.array_equal(out[:P].cpu().numpy(), want)
    assert np.array_equal(mirror[:P].cpu().numpy(), want)
    # weighted (FedBuff) form, same buffers
    s = a.cpu().numpy()
    den = float(np.float32(sum(float(v) for v in s)))
    kx.reduce_mirror(x, K, P, out, mirror, a=a, denom=den)
    torch.cuda.synchronize()
    ref = torch.empty(ld, device=gpu_device)
    kx.reduce(xh.to(gpu_device), K, P, ref, a=a, denom=den, finalize=True)
    torch.cuda.synchronize()
    assert torch.equal(out[:P], ref[:P]) and torch.equal(mirror[:P].cpu(), ref[:P].cpu())


def test_reduce_mirror_rejects_pageable_host_memory(gpu_device):
    from fedscale_amd import kernels as kx

    x = torch.zeros(2, 64)  # pageable: the kernel must never be handed it
    out = torch.zeros(64, device=gpu_device)
    with pytest.raises(ValueError, match="pinned"):
        kx.reduce_mirror(x, 2, 64, out, torch.zeros(64).pin_memory())
    with pytest.raises(ValueError, match="pinned"):
        kx.reduce_mirror(x.to(gpu_device), 2, 64, out, torch.zeros(64))


def _femnist_adapter(gpu_device, extra_int=False):
    from fedscale_amd import synth
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    names, shapes, _ = synth.femnist_cnn_layout()
    g = torch.Generator().manual_seed(3)
    tensors = [torch.randn(s, generator=g) * 0.05 for s in shapes]
    if extra_int:
        names, tensors = names + ["bn.num_batches_tracked"], tensors + [torch.tensor(5)]
    adapter = TorchModelAdapter(StateDictModule(names, tensors), device=gpu_device)
    return names, tensors, adapter, DeviceAggregator(adapter)


def _uploads(names, tensors, K, seed):
    rng = np.random.default_rng(seed)
    ups = []
    for _ in range(K):
        u = {}
        for n, t in zip(names, tensors):
            a = t.numpy()
            u[n] = (np.asarray(a + int(rng.integers(0, 7)), dtype=np.int64) if a.dtype == np.int64 else
                    (a + rng.standard_normal(a.shape).astype(np.float32) * np.float32(0.01)).astype(np.float32))
        ups.append(u)
    return ups


def _spy(monkeypatch):
    from fedscale_amd import _native
    from fedscale_amd import kernels as kx

    calls, real = [], _native.call

    def spy(fn, *args):
        calls.append((fn, args))
        return real(fn, *args)

    monkeypatch.setattr(_native, "call", spy)
    monkeypatch.setattr(kx, "call", spy)
    return calls


def _oracle_round(ups):
    acc = None
    for k, u in enumerate(ups):
        acc = fedavg_step(acc, u, k == 0)
    return fedavg_close(acc, len(ups))


def test_config1_rounds_read_the_mirror_and_write_egress(gpu_device, monkeypatch):
    """Config 1's shape (10 x 24,492): the reduce reads the staging's pinned mirror and writes the new model
    into the egress snapshot; no H2D of the rows, no D2H of the model; get_weights bit-exact every round, and
    a snapshot held across the next round keeps its version's values."""
    names, tensors, adapter, agg = _femnist_adapter(gpu_device)
    calls = _spy(monkeypatch)
    held = None
    for r in range(4):
        ups = _uploads(names, tensors, 10, r)
        del calls[:]
        agg.start_round(10)
        for k, u in enumerate(ups):
            agg.on_result({"client_id": k, "update_weight": u, "moving_loss": 1.0})
        mir = [c for c in calls if c[0] == "fa_reduce_mirror"]
        head = [c for c in calls if c[0] == "fa_reduce"]
        assert len(mir) == 1 and len(head) == 1, [c[0] for c in calls]
        # round 6: the first m arrivals are reduced out of the mirror while the rest arrive (DeviceRound
        # _launch_head: raw chain, no finalize), the finishing launch continues the chain over rows m..9
        from fedscale_amd.round import DeviceRound

        m = min(9, max(1, int(10 * DeviceRound.SPLIT_FRACTION)))  # the head launch's share of the 10 arrivals
        hx, ld = adapter.staging._hx, adapter.staging._hx.shape[1]
        assert head[0][1][0] == hx.data_ptr() and head[0][1][2] == m and head[0][1][8] == 0
        assert mir[0][1][0] == hx.data_ptr() + m * ld * 4, "the reduce did not read the pinned mirror"
        assert mir[0][1][2] == 10 - m and mir[0][1][5] == head[0][1][6], "the finish does not continue the head's chain"
        assert mir[0][1][7] == adapter._snap.buf.f.data_ptr(), "the mean was not written into the snapshot"
        want = _oracle_round(ups)
        assert_state_equal(adapter.get_weights(), want, f"round {r}")
        assert_state_equal(list(agg.model_weights), want, f"model_weights round {r}")
        if held is not None:  # the previous version's snapshot, held by a reader through this round
            snap, prev = held
            assert_state_equal([v.clone() for v in snap.buf.views], prev, f"held snapshot of round {r - 1}")
            adapter._release_host(snap)
        held = (adapter._acquire_host(), want)
    adapter._release_host(held[0])
    # set_weights (no round kernel) falls back to the D2H snapshot and stays exact
    new = [np.asarray(t.numpy() * 2, dtype=np.float32) for t in tensors]
    adapter.set_weights(new)
    assert_state_equal(adapter.get_weights(), new, "after set_weights")


def test_int64_entries_read_from_the_mirror_without_egress_mirror(gpu_device, monkeypatch):
    """A model with an int64 entry: the rows (fp32 bucket and side table) are still read from the pinned
    mirror, the egress takes the D2H path; bit-exact."""
    names, tensors, adapter, agg = _femnist_adapter(gpu_device, extra_int=True)
    calls = _spy(monkeypatch)
    for r in range(2):
        ups = _uploads(names, tensors, 6, 10 + r)
        del calls[:]
        agg.start_round(6)
        for k, u in enumerate(ups):
            agg.on_result({"client_id": k, "update_weight": u, "moving_loss": 1.0})
        red = [c for c in calls if c[0] == "fa_reduce"]
        side = [c for c in calls if c[0] == "fa_side_accumulate"]
        assert len(red) == 1 and red[0][1][0] == adapter.staging._hx.data_ptr()
        assert len(side) == 1 and side[0][1][0] == adapter.staging._hxi.data_ptr()
        want = _oracle_round(ups)
        got = adapter.get_weights()
        assert_state_equal(got[:-1], want[:-1], f"round {r}")
        # load_state_dict of np.asarray(mean, float32) into the int64 entry truncates (torch_model_adapter.py:31-35)
        assert int(got[-1]) == int(np.float32(want[-1])), f"round {r} int64 entry"


def test_fedbuff_small_round_from_the_mirror(gpu_device):
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAsyncAggregator

    names, tensors, adapter, _ = _femnist_adapter(gpu_device)
    agg = DeviceAsyncAggregator(adapter)
    agg.round = 9
    ups = _uploads(names, tensors, 8, 77)
    for k in range(8):
        agg.client_task_model_version[k] = agg.round - k % 5
    agg.start_round(8)
    for k, u in enumerate(ups):
        agg.on_result({"client_id": k, "update_weight": u, "moving_loss": 1.0})
    s = [1 / (1 + (k % 5)) ** 0.5 for k in range(8)]
    got = adapter.get_weights()
    for i in range(len(names)):
        x = np.stack([u[names[i]].reshape(-1) for u in ups])
        assert np.array_equal(got[i].numpy().reshape(-1), fedbuff_flat(x, s)), names[i]


def test_chunked_small_round_keeps_the_h2d_path(gpu_device, monkeypatch):
    """A round that folds a chunk first (capacity < K) reduces its last chunk from the device slots."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator

    names, tensors, adapter, _ = _femnist_adapter(gpu_device)
    agg = DeviceAggregator(adapter)
    agg.device_round_capacity = 4
    calls = _spy(monkeypatch)
    ups = _uploads(names, tensors, 10, 5)
    agg.start_round(10)
    for k, u in enumerate(ups):
        agg.on_result({"client_id": k, "update_weight": u, "moving_loss": 1.0})
    mir = [c for c in calls if c[0] == "fa_reduce_mirror"]
    assert len(mir) == 1 and mir[0][1][0] == adapter.staging.x.data_ptr()
    assert_state_equal(adapter.get_weights(), _oracle_round(ups), "chunked")


def test_pointer_kinds_and_pageable_rejection(gpu_device):
    """fa_pointer_kind tells device, pinned-and-mapped and other host memory apart without launching anything;
    the entry points that may read host memory check it first (pageable memory would fault the GPU)."""
    from fedscale_amd import _native

    lib = _native.load()
    dev = torch.zeros(64, device=gpu_device)
    pinned = torch.zeros(64).pin_memory()
    pageable = np.zeros(64, dtype=np.float32)
    assert lib.fa_pointer_kind(dev.data_ptr()) == 0
    assert lib.fa_pointer_kind(None) == 0
    assert lib.fa_pointer_kind(pinned.data_ptr()) == 1
    assert lib.fa_pointer_kind(pinned.data_ptr() + 64) == 1  # inside the allocation
    assert lib.fa_pointer_kind(pageable.ctypes.data) == -1
    assert lib.fa_pointer_kind(torch.zeros(64).data_ptr()) == -1


@pytest.mark.parametrize("small_finish", [True, False], ids=["finish_small", "finish_general"])
@pytest.mark.parametrize("K", [1, 3, 4, 5, 7, 10, 16])
def test_head_launch_keeps_every_bit(gpu_device, monkeypatch, K, small_finish):
    """Round 6: small zero-copy FedAvg rounds reduce their first arrivals (SPLIT_FRACTION of K) while the rest arrive
    (DeviceRound._launch_head) and finish with the chain continued from that partial sum — through the small-round
    finish or DeviceRound.finalize_mean; the model is the oracle's, bit for bit, and the same as with one finishing
    launch over all rows, for every K (K < 4: no head launch)."""
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from fedscale_amd.round import DeviceRound

    monkeypatch.setattr(TorchModelAdapter, "SMALL_ROUND_FINISH", small_finish)
    got = {}
    for split in (True, False):
        monkeypatch.setattr(DeviceRound, "SPLIT_SMALL_ROUNDS", split)
        names, tensors, adapter, agg = _femnist_adapter(gpu_device)
        for r in range(3):
            ups = _uploads(names, tensors, K, 100 * K + r)
            agg.start_round(K)
            for k, u in enumerate(ups):
                agg.on_result({"client_id": k, "update_weight": u, "moving_loss": 1.0})
            rnd_head = adapter.staging.head_acc is not None
            w = adapter.get_weights()
            assert_state_equal(w, _oracle_round(ups), f"K={K} split={split} round {r}")
            got[(split, r)] = [t.clone() for t in w]
        assert rnd_head == (split and K >= 4)
    for r in range(3):
        for a, b in zip(got[(True, r)], got[(False, r)]):
            assert torch.equal(a, b)


@pytest.mark.parametrize("policy", [None, "fed-yogi"])
def test_apply_round_joins_the_caller_only_when_device_state_is_exposed(gpu_device, monkeypatch, policy):
    """Round 6: apply_round orders the caller's stream after the round (a hipStreamWaitEvent) only when the round
    leaves device state a caller can read through the API (FedYoGi's m_t / v_t); FedAvg's results are read through
    get_weights / model_weights, which wait for the round themselves.  Both stay exact."""
    import argparse

    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from fedscale_amd.state import DeviceStream

    names, tensors, _, _ = _femnist_adapter(gpu_device)
    args = argparse.Namespace(gradient_policy=policy, yogi_eta=3e-3, yogi_tau=1e-8, yogi_beta=0.9, yogi_beta2=0.99)
    adapter = TorchModelAdapter(StateDictModule(names, [t.clone() for t in tensors]), device=gpu_device,
                                optimizer=TorchServerOptimizer(policy, args, gpu_device))
    agg = DeviceAggregator(adapter, args)
    joins, real = [], DeviceStream._exit

    def spy(self, join, done=None):
        joins.append(join)
        return real(self, join, done)

    monkeypatch.setattr(DeviceStream, "_exit", spy)
    ups = _uploads(names, tensors, 6, 9)
    agg.start_round(6)
    for k, u in enumerate(ups[:-1]):
        agg.on_result({"client_id": k, "update_weight": u, "moving_loss": 1.0})
    del joins[:]
    agg.on_result({"client_id": 5, "update_weight": ups[-1], "moving_loss": 1.0})  # the round's apply_round
    assert (True in joins) == (policy == "fed-yogi"), joins
    if policy is None:
        assert_state_equal(adapter.get_weights(), _oracle_round(ups), "FedAvg after an unjoined round")
        m = np.concatenate([np.asarray(w, np.float32).reshape(-1) for w in agg.model_weights])
        want = np.concatenate([w.reshape(-1) for w in _oracle_round(ups)])
        np.testing.assert_array_equal(m, want)
    else:
        y = adapter.optimizer.gradient_controller
        assert torch.isfinite(torch.cat([t.reshape(-1).cpu() for t in y.m_t])).all()  # read on the caller's stream


@pytest.mark.parametrize("seed", range(6))
def test_small_rounds_random_layouts_bit_exact(gpu_device, seed):
    """Small whole-model FedAvg rounds on random layouts (1-6 fp32 tensors, odd sizes, 0-d included) and random K:
    the native staging, the head launch at SPLIT_FRACTION of K and the small-round finish give the oracle's model bit for
    bit, round after round on the same adapter (the staging, the head accumulator and the snapshots reused)."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    rng = np.random.default_rng(1000 + seed)
    T = int(rng.integers(1, 7))
    shapes = [tuple(int(d) for d in rng.integers(1, 60, size=int(rng.integers(0, 4)))) for _ in range(T)]
    names = [f"t{i}" for i in range(T)]
    tensors = [torch.from_numpy(rng.standard_normal(s).astype(np.float32)) for s in shapes]
    adapter = TorchModelAdapter(StateDictModule(names, tensors), device=gpu_device)
    agg = DeviceAggregator(adapter)
    for r in range(3):
        K = int(rng.integers(2, 25))
        ups = _uploads(names, tensors, K, 10 * seed + r)
        agg.start_round(K)
        for k, u in enumerate(ups):
            agg.on_result({"client_id": k, "update_weight": u, "moving_loss": 1.0})
        assert_state_equal(adapter.get_weights(), _oracle_round(ups), f"seed {seed} round {r} K={K}")


def test_small_round_bad_upload_raises_as_before(gpu_device):
    """An upload the native staging does not take is handed to the Python path, which converts or raises exactly as
    before: a wrong shape raises ValueError naming the entry, a wrong dtype TypeError (retrying the slot then works);
    a list upload still gives the oracle's model."""
    names, tensors, adapter, agg = _femnist_adapter(gpu_device)
    ups = _uploads(names, tensors, 4, 77)
    agg.start_round(4)
    bad = dict(ups[0])
    bad[names[2]] = bad[names[2]].reshape(-1)
    with pytest.raises(ValueError, match=names[2]):
        agg.on_result({"client_id": 0, "update_weight": bad, "moving_loss": 1.0})
    agg.model_in_update -= 1  # (the reference would have died here; undo the caller's count to go on)
    bad = dict(ups[0])
    bad[names[0]] = bad[names[0]].astype(np.float16)
    with pytest.raises(TypeError, match=names[0]):
        agg.on_result({"client_id": 0, "update_weight": bad, "moving_loss": 1.0})
    agg.model_in_update -= 1
    agg.on_result({"client_id": 0, "update_weight": list(ups[0].values()), "moving_loss": 1.0})
    for k, u in enumerate(ups[1:], 1):
        agg.on_result({"client_id": k, "update_weight": u, "moving_loss": 1.0})
    assert_state_equal(adapter.get_weights(), _oracle_round(ups), "after refused uploads")
