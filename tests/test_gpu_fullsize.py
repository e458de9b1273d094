"""Parity at BASELINE.json's full sizes (configs 3-5), checked column-sampled.

Every output column depends only on that column of the K client updates, so recomputing a sample of
columns on the host (from the bit-reproducible synthetic generator, fedscale_amd/synth.py) and
comparing bit for bit checks those columns completely; the sample covers the first/last columns, the
float4 tail and the boundaries between the launch levels.  The host side is a plain numpy
restatement of the same fp32 op sequence (IEEE, like the GPU).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sample_cols(P, n=4096, seed=0):
    rng = np.random.default_rng(seed)
    edges = [0, 1, 2, 3, 4, 5, 255, 256, 257, P - 5, P - 4, P - 3, P - 2, P - 1]
    for b in (2_097_152 * 4, 8192 * 4 * 256, 2048 * 4 * 256):  # around launch-level boundaries
        edges += [b - 1, b, b + 1]
    cols = np.unique(np.concatenate([np.array([c for c in edges if 0 <= c < P]), rng.integers(0, P, size=n)]))
    return cols


def _host_seq_sum(seed, K, cols, k0=0, chunk=100):
    from fedscale_amd import synth

    acc = None
    for c0 in range(0, K, chunk):
        xs = synth.host_columns(seed, range(k0 + c0, k0 + min(K, c0 + chunk)), cols)
        for row in xs:
            acc = row.copy() if acc is None else acc + row
    return acc


def test_c3_resnet18_layout_fedavg_k1000(gpu_device):
    """Config 3: 1000 clients x 11,191,242 fp32 (ResNet-18/CIFAR-10 state_dict incl. BN stats)."""
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    K, P, seed = 1000, 11_191_242, 11
    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=seed)
    out = torch.empty(ld, device="cuda")
    kx.reduce(x, K, P, out, denom=float(np.float32(K)), finalize=True)
    cols = _sample_cols(P)
    want = np.divide(_host_seq_sum(seed, K, cols), K)
    np.testing.assert_array_equal(out[torch.from_numpy(cols).cuda()].cpu().numpy(), want)
    del x


def test_headline_fedavg_and_fedbuff_k1000_p25m(gpu_device):
    """The bench headline's exact launch (1000 x 25M fp32, FedAvg mean, the capped-grid V=32 variant) and
    FedBuff's weighted form of it (aggregator.py:497-507, async_aggregator.py:115-137), column-sampled."""
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    K, P, seed = 1000, 25_000_000, 2024
    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=seed)
    out = torch.empty(ld, device="cuda")
    cols = _sample_cols(P, n=2048, seed=2)
    ci = torch.from_numpy(cols).cuda()
    kx.reduce(x, K, P, out, denom=float(np.float32(K)), finalize=True)
    np.testing.assert_array_equal(out[ci].cpu().numpy(), np.divide(_host_seq_sum(seed, K, cols), K))
    # FedBuff: staleness weights 1/sqrt(1 + s_k), s_k = k mod 6, fp32 products added in order
    w = np.asarray([1 / (1 + (k % 6)) ** 0.5 for k in range(K)], dtype=np.float32)
    denom = np.float32(np.sum(w.astype(np.float64)))
    kx.reduce(x, K, P, out, a=torch.from_numpy(w).cuda(), denom=float(denom), finalize=True)
    acc = np.zeros(len(cols), np.float32)
    for c0 in range(0, K, 100):
        for k, row in zip(range(c0, c0 + 100), synth.host_columns(seed, range(c0, c0 + 100), cols)):
            acc = acc + w[k] * row
    np.testing.assert_array_equal(out[ci].cpu().numpy(), np.divide(acc, denom))
    del x


@pytest.mark.parametrize("weighted", [False, True])
def test_reduce_column_windows_every_column(gpu_device, weighted):
    """A bucket long enough for several rounds of the capped grid runs as column windows (fedagg.hip
    FA_WINDOWS); every column, the windows' seams included, equals the host's in-order fp32 chain."""
    from fedscale_amd import kernels as kx
    from fedscale_amd.bucket import round_up

    K, P = 8, 13_000_003
    assert kx.reduce_launches(K, P, weighted=weighted) > 1
    ld = round_up(P, 64)
    rng = np.random.default_rng(7)
    xh = rng.standard_normal((K, ld), dtype=np.float32)
    a = rng.uniform(0.2, 1.0, K).astype(np.float32) if weighted else None
    denom = np.float32(a.astype(np.float64).sum()) if weighted else np.float32(K)
    x = torch.from_numpy(xh).cuda()
    out = torch.empty(ld, device="cuda")
    kx.reduce(x, K, P, out, a=torch.from_numpy(a).cuda() if weighted else None, denom=float(denom), finalize=True)
    acc = xh[0, :P] * a[0] if weighted else xh[0, :P].copy()
    for k in range(1, K):
        acc = acc + (a[k] * xh[k, :P] if weighted else xh[k, :P])
    np.testing.assert_array_equal(out[:P].cpu().numpy(), np.divide(acc, denom))


def test_c4_fedyogi_k1000_p25m(gpu_device):
    """Config 4 (per-GPU shard) over 1000 x 25M, two rounds of state, in both forms the library has:
      * the UNFUSED pair the single-device drop-in runs since round 3 and bench.py times
        (TorchModelAdapter: fa_reduce FA_FINALIZE into the mean, then fa_yogi_step;
        aggregator.py:505-507 -> optimizers.py:43-63 -> yogi.py:15-36);
      * the fused fa_reduce_yogi (the client-sharded SPMD finish, round.py).
    Both bit-exact against the IEEE numpy restatement on sampled columns, and against each other on every
    column."""
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    K, P, seed = 1000, 25_000_000, 44
    ld = round_up(P, 64)
    f = np.float32
    hp = dict(eta=float(f(3e-3)), tau=float(f(1e-8)), beta=float(f(0.9)), omb=float(f(1.0 - 0.9)),
              omb2=float(f(1.0 - 0.99)))
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=seed)
    last = torch.empty(1, ld, device="cuda")
    synth.fill(last, 1, P, seed=seed + 5000, scale_noise=0.0)
    last = last[0]
    last_u = last.clone()  # the unfused chain's own model (each form carries its own state across rounds)
    m, v, out, mean = (torch.empty(ld, device="cuda") for _ in range(4))
    m_u, v_u, out_u, mean_u = (torch.empty(ld, device="cuda") for _ in range(4))
    cols = _sample_cols(P, n=2048, seed=1)
    ci = torch.from_numpy(cols).cuda()
    L = last[ci].cpu().numpy()
    mh = np.zeros(len(cols), f)
    vh = np.full(len(cols), f(hp["tau"]))
    cur = np.divide(_host_seq_sum(seed, K, cols), K)
    for r in range(2):
        # what the drop-in runs (torch_model_adapter.py _apply_yogi): the mean, then the step
        kx.reduce(x, K, P, mean_u, denom=float(f(K)), finalize=True)
        kx.yogi_step(mean_u, last_u, m_u, v_u, out_u, P, init=(r == 0), **hp)
        kx.reduce_yogi(x, K, P, last=last, m=m, v=v, out=out, denom=float(f(K)), init=(r == 0), mean_out=mean, **hp)
        g = cur - L
        g2 = g * g
        mh = f(hp["beta"]) * mh + f(hp["omb"]) * g
        vh = vh - (f(hp["omb2"]) * g2) * np.sign(vh - g2)
        step = ((f(1) / (np.sqrt(vh) + f(hp["tau"]))) * f(hp["eta"])) * mh
        new = L + step
        for got_mean, got_m, got_v, got_out in ((mean_u, m_u, v_u, out_u), (mean, m, v, out)):
            np.testing.assert_array_equal(got_mean[ci].cpu().numpy(), cur)
            np.testing.assert_array_equal(got_m[ci].cpu().numpy(), mh)
            np.testing.assert_array_equal(got_v[ci].cpu().numpy(), vh)
            np.testing.assert_array_equal(got_out[ci].cpu().numpy(), new)
        for a, b in ((mean_u, mean), (m_u, m), (v_u, v), (out_u, out)):  # every column: the two forms agree
            assert torch.equal(a[:P], b[:P])
        last.copy_(out)  # next round starts from the new model
        last_u.copy_(out_u)
        L = new
    del x


def test_c5_qfedavg_shard_k10000_chain_deferred_as_the_drop_in_runs_it(gpu_device):
    """Config 5's per-GPU shard (10,000 x 12.5M, q-FedAvg) exactly as DeviceRound runs it at that K and as
    bench.py times it: chunks of fa_qfed_max_chunk() clients (4 x 2048 + 1808), the fused FedAvg chain
    (``chain=``, the 8-float4 LDS-DMA kernel; aggregator.py:497-507) and a workspace sized for the call's
    (ld, P), so the per-client norm gathers run once per call (deferred).  Delta and chain bit-exact on
    sampled columns, the mean from the chain bit-exact, norms within 1e-9 of the host's fp64 sums, hs and the
    new model bit-exact (optimizers.py:73-104)."""
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    K, P, seed = 10_000, 12_500_000, 56
    chunk = kx.qfed_max_chunk()
    lr, q = 0.05, 1.0
    ld = round_up(P, 64)
    assert kx.qfed_launches(ld, P, chain=True) > 1  # several column windows: the deferred gathers apply
    rng = np.random.default_rng(8)
    losses = rng.uniform(0.5, 2.0, size=K)
    alpha = np.array([np.float32(np.float_power(l + 1e-10, q)) for l in losses], dtype=np.float32)
    x = torch.empty(chunk, ld, device="cuda")
    last = torch.empty(1, ld, device="cuda")
    synth.fill(last, 1, P, seed=seed + 90000, scale_noise=0.0)
    last = last[0]
    delta = torch.zeros(ld, device="cuda")
    chain = torch.zeros(ld, device="cuda")
    sq = torch.zeros(K, dtype=torch.float64, device="cuda")
    ws = kx.qfed_workspace(chunk, "cuda", ld, P)  # DeviceRound._init_qfed's workspace
    al = torch.from_numpy(alpha).cuda()
    bounds = list(range(0, K, chunk)) + [K]
    nch = -(-K // chunk)
    assert len(bounds) - 1 == nch > 1 and bounds[-1] - bounds[-2] == K - (nch - 1) * chunk
    for c, (k0, k1) in enumerate(zip(bounds[:-1], bounds[1:])):
        synth.fill(x, k1 - k0, P, seed=seed, k0=k0)
        kx.qfed_accumulate(x, k1 - k0, P, last=last, alpha=al[k0:k1], lr=lr, delta=delta, sqnorm=sq[k0:k1],
                           workspace=ws, accumulate=c > 0, chain=chain)
    mean = torch.empty(ld, device="cuda")
    kx.reduce(chain.view(1, ld), 1, P, mean, denom=float(np.float32(K)), finalize=True)  # mean_from_staging
    cols = _sample_cols(P, n=1024, seed=3)
    ci = torch.from_numpy(cols).cuda()
    L = last[ci].cpu().numpy()
    d = acc = None
    for c0 in range(0, K, 500):
        for i, row in enumerate(synth.host_columns(seed, range(c0, c0 + 500), cols)):
            g = (L - row) / np.float32(lr)
            t = alpha[c0 + i] * g
            d = t if d is None else d + t
            acc = row.copy() if acc is None else acc + row
    np.testing.assert_array_equal(delta[ci].cpu().numpy(), d)
    np.testing.assert_array_equal(chain[ci].cpu().numpy(), acc)
    np.testing.assert_array_equal(mean[ci].cpu().numpy(), np.divide(acc, np.float32(K)))
    sqh = sq.cpu().numpy()
    allc = np.arange(P)
    Lfull = last[:P].cpu().numpy()
    for k in (0, chunk - 1, chunk, (nch - 1) * chunk + 17, K - 1):  # chunk seams included
        g = (Lfull - synth.host_columns(seed, [k], allc)[0]) / np.float32(lr)
        ref = np.sum((g * g).astype(np.float64))
        assert abs(sqh[k] - ref) <= 1e-9 * ref
    assert np.all(sqh > 0)
    del x
    c1 = np.array([np.float32(q * np.float_power(l + 1e-10, q - 1)) for l in losses], dtype=np.float32)
    c2 = np.array([np.float32((1.0 / lr) * np.float_power(l + 1e-10, q)) for l in losses], dtype=np.float32)
    hs_dev = torch.zeros(2, device="cuda")
    new = torch.empty(ld, device="cuda")
    kx.qfed_hs(sq, torch.from_numpy(c1).cuda(), torch.from_numpy(c2).cuda(), K, hs_dev)
    kx.qfed_finalize(last, delta, hs_dev, new, P)
    hs = np.float32(0.0)
    for k in range(K):
        hs = np.float32(hs + np.float32(c1[k] * np.float32(sqh[k]) + c2[k]))
    hs_got = hs_dev.cpu().numpy()
    assert hs_got[0] == hs and hs_got[1] == np.float32(hs + np.float32(1e-10))
    np.testing.assert_array_equal(new[ci].cpu().numpy(), L - d / np.float32(hs_got[1]))


def test_c5_qfedavg_shard_k10000_streamed(gpu_device):
    """Config 5 per-GPU shard: 10,000 clients x 12.5M (100M / 8 GPUs), q-FedAvg, streamed in chunks of
    1,000 clients through one staging buffer (500 GB of updates never resident at once)."""
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    K, P, seed, chunk = 10_000, 12_500_000, 55, 1000
    lr, q = 0.05, 1.0
    ld = round_up(P, 64)
    rng = np.random.default_rng(7)
    losses = rng.uniform(0.5, 2.0, size=K)
    alpha = np.array([np.float32(np.float_power(l + 1e-10, q)) for l in losses], dtype=np.float32)
    x = torch.empty(chunk, ld, device="cuda")
    last = torch.empty(1, ld, device="cuda")
    synth.fill(last, 1, P, seed=seed + 90000, scale_noise=0.0)  # same base as the clients (seed-independent noise)
    last = last[0]
    delta = torch.zeros(ld, device="cuda")
    sq = torch.zeros(K, dtype=torch.float64, device="cuda")
    ws = kx.qfed_workspace(chunk, "cuda")
    al = torch.from_numpy(alpha).cuda()
    for c in range(K // chunk):
        synth.fill(x, chunk, P, seed=seed, k0=c * chunk)
        kx.qfed_accumulate(x, chunk, P, last=last, alpha=al[c * chunk:(c + 1) * chunk], lr=lr, delta=delta,
                           sqnorm=sq[c * chunk:(c + 1) * chunk], workspace=ws, accumulate=c > 0)
    cols = _sample_cols(P, n=1024, seed=2)
    L = last[torch.from_numpy(cols).cuda()].cpu().numpy()
    d = None
    for c0 in range(0, K, 500):
        xs = synth.host_columns(seed, range(c0, c0 + 500), cols)
        for i, row in enumerate(xs):
            g = (L - row) / np.float32(lr)
            t = alpha[c0 + i] * g
            d = t if d is None else d + t
    np.testing.assert_array_equal(delta[torch.from_numpy(cols).cuda()].cpu().numpy(), d)
    # per-client squared norms over ALL 12.5M columns, for three clients, recomputed on the host
    sqh = sq.cpu().numpy()
    allc = np.arange(P)
    Lfull = last[:P].cpu().numpy()
    for k in (0, 4321, K - 1):
        g = (Lfull - synth.host_columns(seed, [k], allc)[0]) / np.float32(lr)
        ref = np.sum((g * g).astype(np.float64))
        assert abs(sqh[k] - ref) <= 1e-9 * ref  # fp32 partials of 4 squares, then fp64
    assert np.all(sqh > 0)
    del x
    # the round's finish over the whole 10,000-client chain (optimizers.py:96-104): hs from the device's
    # norms with the reference's fp32 recurrence, then new = L - delta / (hs + 1e-10), both bit-exact
    c1 = np.array([np.float32(q * np.float_power(l + 1e-10, q - 1)) for l in losses], dtype=np.float32)
    c2 = np.array([np.float32((1.0 / lr) * np.float_power(l + 1e-10, q)) for l in losses], dtype=np.float32)
    hs_dev = torch.zeros(2, device="cuda")
    new = torch.empty(ld, device="cuda")
    kx.qfed_hs(sq, torch.from_numpy(c1).cuda(), torch.from_numpy(c2).cuda(), K, hs_dev)
    kx.qfed_finalize(last, delta, hs_dev, new, P)
    hs = np.float32(0.0)
    for k in range(K):
        hs = np.float32(hs + np.float32(c1[k] * np.float32(sqh[k]) + c2[k]))
    hs_got = hs_dev.cpu().numpy()
    assert hs_got[0] == hs and hs_got[1] == np.float32(hs + np.float32(1e-10))
    want = L - d / np.float32(hs_got[1])
    np.testing.assert_array_equal(new[torch.from_numpy(cols).cuda()].cpu().numpy(), want)


def test_c2_synthetic_k100_p1m_fedavg_every_column(gpu_device):
    """Config 2 at its exact shape: 100 clients x 1,000,000 fp32, FedAvg, bit-exact on ALL columns against
    the oracle's flat restatement of aggregator.py:497-507 (sequential fp32 sum, true division by K)."""
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up
    from oracle.cpu_reference import fedavg_flat

    K, P, seed = 100, 1_000_000, 22
    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=seed)
    out = torch.empty(ld, device="cuda")
    kx.reduce(x, K, P, out, denom=float(np.float32(K)), finalize=True)
    want = fedavg_flat(x[:, :P].cpu().numpy())
    np.testing.assert_array_equal(out[:P].cpu().numpy(), want)


def test_c2_through_the_drop_in_from_host_updates(gpu_device):
    """Config 2 through the aggregator hook: 100 host uploads of a 1M-parameter model (two tensors, one
    ragged) staged to HBM in chunks of 30 and reduced; the global model is the oracle's mean bit for bit."""
    from fedscale_amd import synth
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from oracle.cpu_reference import fedavg_close, fedavg_step

    K = 100
    names, shapes = ["w", "b"], [(999, 1001), (1_000_000 - 999 * 1001,)]
    model = synth.LayoutModule(names, shapes, [torch.float32, torch.float32])
    agg = DeviceAggregator(TorchModelAdapter(model, device="cuda:0", staging_capacity=30))
    rng = np.random.default_rng(5)
    agg.start_round(K)
    acc = None
    for k in range(K):
        up = {n: rng.standard_normal(s, dtype=np.float32) for n, s in zip(names, shapes)}
        agg.on_result({"client_id": k, "update_weight": up, "moving_loss": 1.0})
        acc = fedavg_step(acc, up, k == 0)
    want = fedavg_close(acc, K)
    for got, w in zip(agg.model_wrapper.get_weights(), want):
        np.testing.assert_array_equal(got.numpy(), w)


@pytest.mark.parametrize("K,P,weighted", [
    (200, 1_000_003, False),    # one round, sw 5 (V = 8 variant), K x sw at the threshold
    (200, 2_300_001, True),     # one round, sw 11 (V = 16), FedBuff weights
    (1000, 3_125_056, False),   # the north star's per-GPU bucket at 8 GPUs (config 4's 25M / 8), sw 14
    (100, 5_000_001, False),    # one round, sw 22 (V = 32)
    (60, 9_000_001, True),      # two rounds of the capped grid at sw 23 (LOOP kernel, run-time width)
])
def test_reduce_balanced_plans_bit_exact(gpu_device, K, P, weighted):
    """The balanced launch plans of fa_reduce (run-time tile width, fedagg.hip launch_plan): every column
    reduced by one thread in arrival order, so bit-exact to the sequential fp32 chain, with the sample
    taken around every tile boundary of the plan."""
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    seed = 300 + K
    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=seed)
    f = np.float32
    w = (np.random.default_rng(K).uniform(0.2, 1.0, size=K).astype(f) if weighted else None)
    out = torch.empty(ld, device="cuda")
    denom = float(f(w.sum())) if weighted else float(f(K))
    kx.reduce(x, K, P, out, a=torch.from_numpy(w).cuda() if weighted else None, denom=denom, finalize=True)
    # tile boundaries of the plan (4 waves x sw strips of 64 float4 per tile)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    S = (ld // 4 + 63) // 64
    gb = cus * 224 // 256
    sw1 = -(-S // (4 * gb))
    if sw1 > 32:
        cap = cus * 75 // 100
        R = -(-S // (4 * 32 * cap))
        sw = -(-S // (4 * R * cap))
    else:
        sw = sw1
    span = 4 * sw * 64 * 4  # floats per tile
    bounds = np.arange(span, P, span)
    cols = np.unique(np.concatenate([_sample_cols(P, n=2048, seed=K),
                                     np.clip(np.concatenate([bounds - 1, bounds]), 0, P - 1)]))
    acc = None
    for c0 in range(0, K, 100):
        xs = synth.host_columns(seed, range(c0, min(K, c0 + 100)), cols)
        for i, row in enumerate(xs):
            k = c0 + i
            t = row * w[k] if weighted else row
            acc = t if acc is None else acc + t
    want = np.divide(acc, f(denom))
    np.testing.assert_array_equal(out[torch.from_numpy(cols).cuda()].cpu().numpy(), want)
    del x


@pytest.mark.parametrize("K,P", [(200, 2_300_001), (150, 5_000_001), (1000, 3_125_056)])
def test_reduce_yogi_balanced_plans_bit_exact(gpu_device, K, P):
    """The fused FedYoGi epilogue on the balanced plans' run-time-width tiles (V = 16 and V = 32 variants
    with sw < V): mean, m, v and the new model bit-exact to the IEEE numpy restatement, two rounds."""
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    seed = 700 + K
    ld = round_up(P, 64)
    f = np.float32
    hp = dict(eta=float(f(3e-3)), tau=float(f(1e-8)), beta=float(f(0.9)), omb=float(f(1.0 - 0.9)),
              omb2=float(f(1.0 - 0.99)))
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=seed)
    last = torch.empty(1, ld, device="cuda")
    synth.fill(last, 1, P, seed=seed + 5000, scale_noise=0.0)
    last = last[0]
    m, v, out, mean = (torch.empty(ld, device="cuda") for _ in range(4))
    cols = _sample_cols(P, n=2048, seed=K)
    ci = torch.from_numpy(cols).cuda()
    L = last[ci].cpu().numpy()
    mh = np.zeros(len(cols), f)
    vh = np.full(len(cols), f(hp["tau"]))
    cur = np.divide(_host_seq_sum(seed, K, cols), K)
    for r in range(2):
        kx.reduce_yogi(x, K, P, last=last, m=m, v=v, out=out, denom=float(f(K)), init=(r == 0), mean_out=mean, **hp)
        g = cur - L
        g2 = g * g
        mh = f(hp["beta"]) * mh + f(hp["omb"]) * g
        vh = vh - (f(hp["omb2"]) * g2) * np.sign(vh - g2)
        new = L + ((f(1) / (np.sqrt(vh) + f(hp["tau"]))) * f(hp["eta"])) * mh
        np.testing.assert_array_equal(mean[ci].cpu().numpy(), cur)
        np.testing.assert_array_equal(m[ci].cpu().numpy(), mh)
        np.testing.assert_array_equal(v[ci].cpu().numpy(), vh)
        np.testing.assert_array_equal(out[ci].cpu().numpy(), new)
        last.copy_(out)
        L = new
    del x


def test_c5_one_gpu_bench_shape_k2c17_p100m(gpu_device):
    """config 5 on ONE GPU exactly as bench.py times it (``Workload`` of c5_qfedavg_k10000_p100M):
    100 M columns, the resident chunk C the bench picks on this box (0.6 of the free HBM, ≈ 462 clients), K = 2C + 17
    so the round streams three passes over the chunk (two full, one of 17), the fused FedAvg chain
    (aggregator.py:497-507) and a workspace holding every column window's partials, so the per-client norms are
    gathered once per call by k_qfed_gather_win_wave over ≈ 50 windows.  Against the oracle's op order
    (optimizers.py:73-104): delta, chain, the mean from the chain and the new model bit-exact on sampled columns that
    include both sides of every chain-window seam; the norms within 1e-9 of fp64 sums over all 100 M columns (the
    clients of the first, a middle and the last row); hs bit-exact (the fp32 recurrence of :96-98)."""
    import bench
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up
    from fedscale_amd.state import ShardGroup

    torch.cuda.empty_cache()
    P, seed, lr = 100_000_000, 2024, 0.05
    ld = round_up(P, 64)
    free, _ = torch.cuda.mem_get_info(gpu_device)
    C = min(max(1, int(free * bench.MEM_FRACTION) // (4 * ld)), kx.qfed_max_chunk())
    assert C >= 64, f"only {C} resident clients fit"
    K = 2 * C + 17
    w = bench.Workload("qfedavg", K, P, 0, 1, gpu_device, seed, ShardGroup(0, 1), chunk=C,
                       budget_fraction=bench.MEM_FRACTION)
    assert w.C == C and len(w.passes) == 3 and w.passes[-1] == (2 * C, 17)
    assert w.mean_chain and w.qf["chain"] is not None  # several passes: the drop-in's fused chain
    win = kx.qfed_window(chain=True)
    nwin = kx.qfed_launches(ld, P, chain=True)
    assert nwin >= 40  # ≈ 50 column windows per call, gathered once per call
    assert w.qf["ws"].numel() * 8 >= _native_ws_bytes(C, ld, P)
    w.step()
    torch.cuda.synchronize()
    qf = w.qf
    seams = np.arange(win, P, win)
    cols = np.unique(np.concatenate([_sample_cols(P, n=1024, seed=5), seams - 1, seams]))
    ci = torch.from_numpy(cols).to(gpu_device)
    L = synth.host_columns(seed, [0], cols, scale_noise=0.0)[0]  # Workload's last: base only
    np.testing.assert_array_equal(qf["last"][ci].cpu().numpy(), L)
    rows = synth.host_columns(seed, range(C), cols)  # the resident chunk (client k of the round reads row k % C)
    alpha = qf["alpha"].cpu().numpy()
    f32 = np.float32
    d = acc = None
    for k in range(K):
        row = rows[k % C]
        g = (L - row) / f32(lr)
        t = alpha[k] * g
        d = t if d is None else d + t
        acc = row.copy() if acc is None else acc + row
    np.testing.assert_array_equal(qf["delta"][ci].cpu().numpy(), d)
    np.testing.assert_array_equal(qf["chain"][ci].cpu().numpy(), acc)
    mean = torch.empty(ld, device=gpu_device)
    kx.reduce(qf["chain"].view(1, ld), 1, P, mean, denom=float(f32(K)), finalize=True)  # mean_from_staging
    np.testing.assert_array_equal(mean[ci].cpu().numpy(), np.divide(acc, f32(K)))
    sq = qf["sq"].cpu().numpy()
    assert np.all(sq > 0)
    for k in range(C):  # a row read in every pass gives its clients the same norm, bit for bit
        assert sq[k] == sq[k + C] and (k >= 17 or sq[k] == sq[k + 2 * C])
    Lfull = qf["last"][:P].cpu().numpy()
    for j in (0, C // 2, C - 1):
        row = w.xs[0][j, :P].cpu().numpy()
        np.testing.assert_array_equal(row[cols], rows[j])
        g = (Lfull - row) / f32(lr)
        ref = np.sum((g * g).astype(np.float64))
        assert abs(sq[j] - ref) <= 1e-9 * ref, (j, sq[j], ref)
        del row, g
    c1, c2 = qf["c1"].cpu().numpy(), qf["c2"].cpu().numpy()
    hs = f32(0.0)
    for k in range(K):
        hs = f32(hs + f32(c1[k] * f32(sq[k]) + c2[k]))
    hs_got = qf["hs"].cpu().numpy()
    assert hs_got[0] == hs and hs_got[1] == f32(hs + f32(1e-10))
    np.testing.assert_array_equal(w.out[ci].cpu().numpy(), L - d / f32(hs_got[1]))
    w.free()
    del mean


def _native_ws_bytes(K, ld, P):
    from fedscale_amd import _native

    return int(_native.load().fa_qfed_workspace_bytes(K, ld, P))
