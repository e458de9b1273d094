"""World-size-2 tests of the sharded (one process per GPU) path, gloo backend, 127.0.0.1."""
import socket

import pytest
import torch.multiprocessing as mp

from tests import dist_workers
from tests.golden_io import scenario_names


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("name", ["fedavg_femnist_cnn_k10", "fedavg_mixed_k7", "fedavg_wide_k64"])
def test_cpu_sharded_reduction_world2(name):
    mp.spawn(dist_workers.cpu_shard_worker, args=(2, _port(), name), nprocs=2, join=True)


@pytest.mark.parametrize("name", ["fedavg_femnist_cnn_k10"])
def test_cpu_sharded_reduction_world3(name):
    mp.spawn(dist_workers.cpu_shard_worker, args=(3, _port(), name), nprocs=3, join=True)


@pytest.mark.parametrize("name,world", [("fedavg_femnist_cnn_k10", 2), ("fedavg_mixed_k7", 2),
                                        ("fedavg_wide_k64", 2), ("fedavg_mixed_k3", 3), ("fedavg_wide_k64", 4)])
def test_cpu_client_sharded_reduction(name, world):
    mp.spawn(dist_workers.cpu_client_shard_worker, args=(world, _port(), name), nprocs=world, join=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name", [n for n in scenario_names() if n != "kat_linear_225"])
def test_gpu_sharded_device_path_world2(gpu_device, name):
    mp.spawn(dist_workers.gpu_shard_worker, args=(2, _port(), name, 2), nprocs=2, join=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name", [n for n in scenario_names() if n != "kat_linear_225"])
def test_gpu_client_sharded_device_path_world2(gpu_device, name):
    mp.spawn(dist_workers.gpu_shard_worker, args=(2, _port(), name, 2, "clients"), nprocs=2, join=True)


@pytest.mark.parametrize("name", ["fedavg_wide_k64", "fedavg_femnist_cnn_k10"])
def test_cpu_sharded_reduction_world8(name):
    """Eight ranks (BASELINE config 5's 8-way split): balanced 64-aligned slices, the all-gather reassembles the
    unsharded mean bit for bit, and the fixed-order norm exchange matches on every rank."""
    mp.spawn(dist_workers.cpu_shard_worker, args=(8, _port(), name), nprocs=8, join=True)


@pytest.mark.parametrize("name", ["fedavg_wide_k64", "fedavg_femnist_cnn_k10"])
def test_cpu_client_sharded_reduction_world8(name):
    mp.spawn(dist_workers.cpu_client_shard_worker, args=(8, _port(), name), nprocs=8, join=True)


def test_rccl_probe_skips_on_every_rank_together():
    mp.spawn(dist_workers.rccl_probe_agreement_worker, args=(3, _port(), 1), nprocs=3, join=True)


def test_rccl_probe_failing_rank_does_not_hang_the_others():
    mp.spawn(dist_workers.rccl_probe_failure_worker, args=(3, _port(), 1), nprocs=3, join=True)


def test_rccl_probe_gathers_every_ranks_view():
    mp.spawn(dist_workers.rccl_probe_success_worker, args=(2, _port()), nprocs=2, join=True)
