"""Worker functions for the multi-process tests (spawned; importable module)."""
import os

import numpy as np
import torch
import torch.distributed as dist


def _init(rank, world, port):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)


def cpu_shard_worker(rank, world, port, name):
    """Sharded layout + collectives on CPU: every rank reduces its slice with the oracle arithmetic;
    the all-gather reassembles exactly the unsharded result, and the all-reduced per-client partial
    squared norms equal the unsharded ones (the q-FedAvg exchange)."""
    from fedscale_amd.bucket import BucketLayout
    from fedscale_amd.state import ShardGroup
    from oracle.cpu_reference import fedavg_flat
    from tests.golden_io import Scenario

    _init(rank, world, port)
    try:
        sc = Scenario(name)
        dtypes = [getattr(torch, d) for d in sc.meta["dtypes"]]
        full = BucketLayout(sc.names, sc.meta["shapes"], dtypes)
        lay = BucketLayout(sc.names, sc.meta["shapes"], dtypes, rank, world)
        K = sc.meta["rounds"][0]
        xs = np.zeros((K, lay.ld), np.float32)
        xf = np.zeros((K, full.ld), np.float32)
        for k in range(K):
            upd = full.values_of(sc.client(k))
            lay.pack_host(upd, xs[k], np.zeros(lay.ldq, np.int64))
            full.pack_host(upd, xf[k], np.zeros(full.ldq, np.int64))
        g = ShardGroup(rank, world)
        shard_mean = fedavg_flat(xs[:, :lay.ld]) if K > 0 else None
        gathered = g.all_gather(torch.from_numpy(shard_mean)).numpy()
        np.testing.assert_array_equal(lay.unshard(gathered), fedavg_flat(xf)[:full.P_full])
        # the slices tile [0, P) in rank order, 64-aligned, each within 64 floats of P/world, every row ld wide
        sizes = g.collective_all_gather(torch.tensor([lay.p0, lay.p1, lay.ld])).numpy().reshape(world, 3)
        assert sizes[0, 0] == 0 and sizes[-1, 1] == full.P_full and (sizes[1:, 0] == sizes[:-1, 1]).all()
        assert (sizes[:, 0] % 64 == 0).all() and (sizes[:, 2] == lay.ld).all()
        if full.P_full >= 64 * world:
            assert (np.abs((sizes[:, 1] - sizes[:, 0]) - full.P_full / world) <= 64).all()
        # q-FedAvg partial norms
        L = xf[0] * np.float32(0.5)
        Ls = L[lay.p0:lay.p0 + lay.ld] if lay.P else np.zeros(lay.ld, np.float32)
        Ls = np.pad(Ls, (0, lay.ld - len(Ls)))
        part = np.array([np.sum(((Ls[:lay.P] - xs[k, :lay.P]) / np.float32(0.05)) ** 2, dtype=np.float64)
                         for k in range(K)])
        tot = g.all_reduce_sum(torch.from_numpy(part.copy())).numpy()
        want = np.array([np.sum(((L[:full.P_full] - xf[k, :full.P_full]) / np.float32(0.05)) ** 2,
                                dtype=np.float64) for k in range(K)])
        np.testing.assert_allclose(tot, want, rtol=1e-12)
        # the same exchange in a fixed rank order (ShardGroup.sum_partials): ((p_0 + p_1) + p_2) + ... on
        # every rank, bit for bit, whatever order the transport combines in
        fixed = g.sum_partials(torch.from_numpy(part.copy())).numpy()
        parts = g.collective_all_gather(torch.from_numpy(part.copy())).numpy().reshape(world, K)
        acc = parts[0].copy()
        for r in range(1, world):
            acc = acc + parts[r]
        np.testing.assert_array_equal(fixed, acc)
        everyone = g.collective_all_gather(torch.from_numpy(fixed.copy())).numpy().reshape(world, K)
        assert (everyone == everyone[0]).all()
        np.testing.assert_allclose(fixed, want, rtol=1e-12)
    finally:
        dist.destroy_process_group()


def cpu_client_shard_worker(rank, world, port, name):
    """Client mode on CPU: every rank reduces its contiguous block of arrivals with the oracle chain, the
    all-reduced partial chains / K equal the unsharded FedAvg mean within fp32 re-association error, and
    the int64 side-table sums are exact."""
    from fedscale_amd.bucket import BucketLayout
    from fedscale_amd.state import ShardGroup
    from oracle.cpu_reference import fedavg_flat
    from tests.golden_io import Scenario

    _init(rank, world, port)
    try:
        sc = Scenario(name)
        dtypes = [getattr(torch, d) for d in sc.meta["dtypes"]]
        full = BucketLayout(sc.names, sc.meta["shapes"], dtypes)
        K = sc.meta["rounds"][0]
        g = ShardGroup(rank, world, mode="clients")
        k0, k1 = g.client_block(K)
        assert all(g.owner(k, K) == rank for k in range(k0, k1))
        xf = np.zeros((K, full.ld), np.float32)
        xi = np.zeros((K, full.ldq), np.int64)
        for k in range(K):
            full.pack_host(full.values_of(sc.client(k)), xf[k], xi[k])
        part = np.zeros(full.ld, np.float32)
        for k in range(k0, k1):  # the rank's own chain, from its first client
            part = xf[k].copy() if k == k0 else part + xf[k]
        tot = g.all_reduce_sum(torch.from_numpy(part)).numpy() / np.float32(K)
        want = fedavg_flat(xf)
        np.testing.assert_allclose(tot[:full.P_full], want[:full.P_full], rtol=1e-5,
                                   atol=1e-6 * float(np.abs(want).max() + 1e-30))
        side = g.all_reduce_sum(torch.from_numpy(xi[k0:k1].sum(axis=0))).numpy()
        np.testing.assert_array_equal(side, xi.sum(axis=0))
    finally:
        dist.destroy_process_group()


def gpu_shard_worker(rank, world, port, name, capacity, mode="params"):
    """The full device path with the round spread over `world` ranks (all on cuda:0, gloo for the
    collectives).  mode "params": per-shard kernels, q-FedAvg norm all-reduce, all-gather reassembly on
    egress (bit-exact).  mode "clients": per-rank blocks of arrivals, all-reduced partials, replicated
    server step (within the north-star tolerance)."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator, DeviceAsyncAggregator
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from fedscale_amd.state import ShardGroup
    from tests.golden_io import Scenario, StateDictModule, assert_state_close, assert_state_equal

    _init(rank, world, port)
    torch.cuda.set_device(0)
    try:
        sc = Scenario(name)
        args = sc.args()
        opt = (TorchServerOptimizer(args.gradient_policy, args, "cuda:0")
               if sc.meta.get("optimizer") is not None else None)
        adapter = TorchModelAdapter(StateDictModule(sc.names, sc.init_state()), optimizer=opt, device="cuda:0",
                                    shards=ShardGroup(rank, world, mode=mode), staging_capacity=capacity)
        policy = sc.meta["policy"]
        if policy == "fedbuff":
            agg = DeviceAsyncAggregator(adapter, args)
            agg.round = sc.meta["round"]
            for k, s in enumerate(sc.meta["staleness"]):
                agg.client_task_model_version[101 + k] = agg.round - s
        else:
            agg = DeviceAggregator(adapter, args)
        for r, ks in sc.rounds():
            if policy == "q-fedavg":
                args.learning_rate = sc.meta["lrs"][r]
            agg.start_round(len(ks))
            for res in sc.results(ks, r):
                agg.on_result(res)
            got = adapter.get_weights()
            if mode == "clients":  # re-associated fp32 sums; int64 FedAvg sums stay exact
                assert_state_close(got, sc.expected(r), 1e-5, f"{name} clients rank{rank} r{r}",
                                   int_slack=0 if policy == "fedavg" and opt is None else 1)
            elif policy == "q-fedavg":
                assert_state_close(got, sc.expected(r), 1e-5, f"{name} rank{rank} r{r}", int_slack=1)
            elif policy == "fed-yogi":
                assert_state_close(got, sc.expected(r), 1e-6, f"{name} rank{rank} r{r}")
            else:
                assert_state_equal(got, sc.expected(r), f"{name} rank{rank} r{r}")
    finally:
        dist.destroy_process_group()


def rccl_probe_agreement_worker(rank, world, port, unavailable_rank):
    """spmd_rccl_probe on CPU ranks: when RCCL cannot be loaded on one rank, EVERY rank returns "skipped" together
    (none enters the blocking ncclCommInitRank alone)."""
    from fedscale_amd import _native
    from fedscale_amd.state import spmd_rccl_probe

    _init(rank, world, port)
    try:
        lib = _native.load()
        real = lib.fa_rccl_available

        class _Lib:
            def __getattr__(self, name):
                return getattr(lib, name)

            @staticmethod
            def fa_rccl_available():
                return 0 if rank == unavailable_rank else real()

        orig = _native.load
        _native.load = lambda *a, **k: _Lib()
        try:
            r = spmd_rccl_probe(0)
        finally:
            _native.load = orig
        assert "skipped" in r and str(unavailable_rank) in r["skipped"], r
    finally:
        dist.destroy_process_group()


def rccl_probe_failure_worker(rank, world, port, failing_rank):
    """spmd_rccl_probe when ONE rank's ncclCommInitRank fails or hangs.  Each rank's part runs in a child
    process under a deadline; here the child is simulated (the CPU has no GPU): the failing rank's times out, the
    others report success.  Every rank must return — none blocks in a collective the failing rank never enters — and
    every rank must name the failing rank."""
    import json
    import subprocess

    from fedscale_amd import _native
    from fedscale_amd.state import spmd_rccl_probe

    _init(rank, world, port)
    try:
        lib = _native.load()

        class _Lib:
            def __getattr__(self, name):
                return getattr(lib, name)

            @staticmethod
            def fa_rccl_available():
                return 1

        orig_load, orig_call, orig_run = _native.load, _native.call, subprocess.run

        def call(name, *a):
            if name == "fa_rccl_unique_id":
                return 0  # the id buffer stays zeros: the simulated children never read it
            return orig_call(name, *a)

        def run(cmd, **kw):
            assert "fedscale_amd.rccl_probe" in cmd and kw.get("timeout"), cmd
            if rank == failing_rank:
                raise subprocess.TimeoutExpired(cmd, kw["timeout"])
            out = {"rank": rank, "ok": True, "count": world, "user_rank": rank, "cu_device": rank}
            return subprocess.CompletedProcess(cmd, 0, json.dumps(out) + "\n", "")

        _native.load, _native.call, subprocess.run = (lambda *a, **k: _Lib()), call, run
        try:
            r = spmd_rccl_probe(rank, timeout_s=5)
        finally:
            _native.load, _native.call, subprocess.run = orig_load, orig_call, orig_run
        assert "error" in r and list(r["rank_errors"]) == [failing_rank], r
        assert "no result within" in r["rank_errors"][failing_rank], r
    finally:
        dist.destroy_process_group()


def rccl_probe_success_worker(rank, world, port):
    """spmd_rccl_probe with every (simulated) child succeeding: every rank gets the same table of RCCL's view."""
    import json
    import subprocess

    from fedscale_amd import _native
    from fedscale_amd.state import spmd_rccl_probe

    _init(rank, world, port)
    try:
        lib = _native.load()

        class _Lib:
            def __getattr__(self, name):
                return getattr(lib, name)

            @staticmethod
            def fa_rccl_available():
                return 1

        orig_load, orig_call, orig_run = _native.load, _native.call, subprocess.run

        def call(name, *a):
            return 0 if name == "fa_rccl_unique_id" else orig_call(name, *a)

        def run(cmd, **kw):
            out = {"rank": rank, "ok": True, "count": world, "user_rank": rank, "cu_device": rank}
            return subprocess.CompletedProcess(cmd, 0, json.dumps(out) + "\n", "")

        _native.load, _native.call, subprocess.run = (lambda *a, **k: _Lib()), call, run
        try:
            r = spmd_rccl_probe(rank, timeout_s=5)
        finally:
            _native.load, _native.call, subprocess.run = orig_load, orig_call, orig_run
        assert r["count"] == world and r["counts_agree"] and r["rank_of_process"] == list(range(world)), r
    finally:
        dist.destroy_process_group()
