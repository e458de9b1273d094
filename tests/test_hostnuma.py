"""Host NUMA binding of the staging thread (fedscale_amd/hostnuma.py), with the topology mocked (CPU only)."""
import pytest

from fedscale_amd import hostnuma


def test_cpulist_parsing():
    assert hostnuma._cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert hostnuma._cpulist("") == set()


@pytest.fixture
def two_nodes(monkeypatch):
    calls = []
    monkeypatch.setattr(hostnuma.glob, "glob", lambda pat: ["/sys/devices/system/node/node0",
                                                            "/sys/devices/system/node/node1"])
    monkeypatch.setattr(hostnuma, "node_cpus", lambda n: {0: {0, 1, 2, 3}, 1: {4, 5, 6, 7}}[n])
    monkeypatch.setattr(hostnuma.os, "sched_getaffinity", lambda pid: {2, 3, 4, 5})
    monkeypatch.setattr(hostnuma.os, "sched_setaffinity", lambda pid, cpus: calls.append(set(cpus)))
    return calls


def test_binds_to_the_gpus_node_within_the_allowed_cpus(two_nodes, monkeypatch):
    monkeypatch.setattr(hostnuma, "gpu_numa_node", lambda d: 1)
    assert hostnuma.bind_to_gpu("cuda:0") == 1
    assert two_nodes == [{4, 5}]


def test_no_change_without_a_node_or_allowed_cpus(two_nodes, monkeypatch):
    monkeypatch.setattr(hostnuma, "gpu_numa_node", lambda d: None)
    assert hostnuma.bind_to_gpu("cuda:0") is None
    monkeypatch.setattr(hostnuma, "node_cpus", lambda n: {9})
    monkeypatch.setattr(hostnuma, "gpu_numa_node", lambda d: 0)
    assert hostnuma.bind_to_gpu("cuda:0") is None
    assert two_nodes == []


def test_single_node_host_is_left_alone(monkeypatch):
    monkeypatch.setattr(hostnuma.glob, "glob", lambda pat: ["/sys/devices/system/node/node0"])
    monkeypatch.setattr(hostnuma.os, "sched_setaffinity", lambda pid, cpus: pytest.fail("must not bind"))
    assert hostnuma.bind_to_gpu("cuda:0") is None


def test_no_gpu_means_no_node():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    assert hostnuma.gpu_numa_node("cuda:0") is None


def test_binding_lowers_torch_threads_to_the_node(two_nodes, monkeypatch):
    """threads started after the binding inherit it, so torch's pool is cut to the node's CPUs."""
    import torch

    monkeypatch.setattr(hostnuma, "gpu_numa_node", lambda d: 1)
    set_calls = []
    monkeypatch.setattr(torch, "get_num_threads", lambda: 16)
    monkeypatch.setattr(torch, "set_num_threads", lambda n: set_calls.append(n))
    assert hostnuma.bind_to_gpu("cuda:0", match_torch_threads=True, log=True) == 1
    assert two_nodes == [{4, 5}] and set_calls == [2]


def test_mixin_numa_binding_is_opt_in():
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregatorMixin

    assert DeviceAggregatorMixin.device_numa_bind is False
