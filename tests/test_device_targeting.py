"""CPU checks of device targeting (no GPU here: torch.cuda is replaced by a model of N devices with
per-device current streams and a current device, as HIP and torch keep them per thread).

What they pin:
* ``DeviceStream`` makes its GPU current and its own (non-null) stream current on it for the span of a
  ``with``, whatever device the caller had current, and restores both; ``joined()`` orders the caller's
  stream after the work; ``wait_caller()`` orders the stream after the OUTERMOST caller's stream;
* ``DeviceGroup``'s RCCL stream tables hold each position's own stream (never ``current_stream(d)``, whose
  handle is 0 for torch's default stream, i.e. HIP's null stream of whatever device is current);
* the aggregator mixin builds its adapter on the reference's ``self.device`` (``--cuda_device``,
  aggregator.py:47) and refuses a CPU device.
The GPU side of the same contract (every native call of every part carries that part's stream) is
``tests/test_gpu_sharded.py::test_every_native_call_runs_on_its_parts_stream``."""
import argparse
import itertools

import pytest
import torch


class FakeStream:
    _ids = itertools.count(0x1000, 0x100)

    def __init__(self, dev: int, handle=None):
        self.device_index = dev
        self.device = torch.device("cuda", dev)
        self.device_type = 1
        self.cuda_stream = next(self._ids) if handle is None else handle
        self.stream_id = self.cuda_stream
        self.waited = []

    def wait_stream(self, other):
        self.waited.append(other)

    def wait_event(self, ev):
        self.waited.append(ev.src)


class FakeEvent:
    def __init__(self, *a, **k):
        self.src = None

    def record(self, stream=None):
        self.src = stream


class FakeCuda:
    """torch.cuda as seen by one thread: a current device and a current stream per device (the state.py
    helpers that read and set them are replaced)."""

    def __init__(self, monkeypatch, ndev: int, current: int = 0):
        from fedscale_amd import state

        self.cur = current
        self.ndev = ndev
        self.default = {d: FakeStream(d, 0) for d in range(ndev)}  # torch's default stream: handle 0
        self.stream_of = dict(self.default)
        self.by_key = {state._stream_key(s): s for s in self.default.values()}
        monkeypatch.setattr(state, "_get_device", lambda: self.cur)
        monkeypatch.setattr(state, "_set_device", self.set_device)
        monkeypatch.setattr(state, "_get_stream", lambda i: state._stream_key(self.stream_of[i]))
        monkeypatch.setattr(state, "_set_stream", lambda key: self.set_stream(self.by_key[key]))
        monkeypatch.setattr(state, "_stream_obj", lambda key: self.by_key[key])
        monkeypatch.setattr(torch.cuda, "current_stream", self.current_stream)
        monkeypatch.setattr(torch.cuda, "Stream", self.new_stream)
        monkeypatch.setattr(torch.cuda, "Event", FakeEvent)

    def set_device(self, d):
        assert 0 <= int(d) < self.ndev
        self.cur = int(d)

    def current_stream(self, d=None):
        return self.stream_of[self.cur if d is None else (d.index if isinstance(d, torch.device) else int(d))]

    def set_stream(self, s):
        self.stream_of[s.device_index] = s

    def new_stream(self, device=None):
        from fedscale_amd import state

        s = FakeStream(torch.device(device).index)
        self.by_key[state._stream_key(s)] = s
        return s

    def adopt(self, s):
        from fedscale_amd import state

        self.by_key[state._stream_key(s)] = s
        return s


def test_device_stream_targets_its_device_whatever_is_current(monkeypatch):
    from fedscale_amd.state import DeviceStream

    fc = FakeCuda(monkeypatch, 4, current=0)
    parts = [DeviceStream(d) for d in range(4)]
    assert all(p.handle != 0 for p in parts), "a part's stream is never the null stream"
    assert len({p.handle for p in parts}) == 4
    fc.cur = 2  # the caller has another GPU current
    for p in parts:
        with p:
            assert fc.cur == p.index
            assert torch.cuda.current_stream(p.index) is p.stream
            assert DeviceStream.current() is p
        assert fc.cur == 2 and DeviceStream.current() is None
        assert torch.cuda.current_stream(p.index) is fc.default[p.index]
    # nesting across devices (the coordinator of a sharded model calls into parts)
    with parts[1]:
        with parts[3]:
            assert fc.cur == 3 and DeviceStream.current() is parts[3]
        assert fc.cur == 1 and torch.cuda.current_stream(1) is parts[1].stream
    assert fc.cur == 2


def test_device_stream_joined_and_wait_caller(monkeypatch):
    from fedscale_amd.state import DeviceStream

    fc = FakeCuda(monkeypatch, 2, current=1)
    caller = fc.adopt(FakeStream(0))
    fc.stream_of[0] = caller  # the caller works on its own stream of device 0
    ds = DeviceStream(0)
    with ds.joined():
        with ds:  # nested entry of the same part: its "previous" stream is ds itself
            ds.wait_caller()
        assert ds.stream.waited == [caller], "wait_caller must wait for the outermost caller's stream"
    assert caller.waited == [ds.stream], "joined(): the caller's stream waits for the part's work"
    assert fc.cur == 1 and torch.cuda.current_stream(0) is caller
    with ds:
        pass
    assert caller.waited == [ds.stream], "a plain entry does not join"


def test_device_group_stream_tables_hold_each_positions_stream(monkeypatch):
    from fedscale_amd.state import DeviceGroup

    fc = FakeCuda(monkeypatch, 8, current=5)
    g = DeviceGroup(list(range(8)), transport="copy")  # "copy": no RCCL needed to build the tables
    fake = [torch.empty(0)] * 8
    monkeypatch.setattr(torch.Tensor, "data_ptr", lambda self: 0x10000, raising=False)
    (send,), streams = g._tables(fake)
    hs = list(streams)
    assert hs == g.stream_handles() == [ds.handle for ds in g.streams]
    assert all(h for h in hs) and len(set(hs)) == 8
    assert [ds.index for ds in g.streams] == list(range(8))
    assert fc.cur == 5


def test_device_group_rejects_bad_device_lists():
    from fedscale_amd.state import DeviceGroup

    with pytest.raises(ValueError, match="indexed GPUs"):
        DeviceGroup(["cpu"])
    with pytest.raises(ValueError, match="at least one"):
        DeviceGroup([])


class _Wrapper:
    def __init__(self, model):
        self.model = model

    def get_model(self):
        return self.model


class _RefAggregator:
    """Stands for the reference Aggregator's init_model (aggregator.py:198-211): a model wrapper."""

    def init_model(self):
        self.model_wrapper = _Wrapper(torch.nn.Linear(3, 2))


@pytest.mark.parametrize("cuda_device, want", [("cuda:3", torch.device("cuda", 3)), (None, None),
                                                (torch.device("cuda:1"), torch.device("cuda", 1))])
def test_mixin_builds_the_adapter_on_the_reference_device(monkeypatch, cuda_device, want):
    from fedscale_amd.cloud.aggregation import aggregator as aggmod

    seen = {}

    class Recorder:
        def __init__(self, model, optimizer=None, device=None):
            seen["device"], seen["opt_device"] = device, optimizer.device

    monkeypatch.setattr(aggmod, "TorchModelAdapter", Recorder)
    monkeypatch.delenv("FEDAGG_DEVICES", raising=False)

    class A(aggmod.DeviceAggregatorMixin, _RefAggregator):
        pass

    a = A()
    a.args = argparse.Namespace(gradient_policy=None)
    a.device = cuda_device  # aggregator.py:47: args.cuda_device if args.use_cuda
    a.init_model()
    assert seen["device"] == want and seen["opt_device"] == want


def test_mixin_refuses_a_cpu_aggregator_device(monkeypatch):
    from fedscale_amd.cloud.aggregation import aggregator as aggmod

    monkeypatch.delenv("FEDAGG_DEVICES", raising=False)

    class A(aggmod.DeviceAggregatorMixin, _RefAggregator):
        pass

    a = A()
    a.args = argparse.Namespace(gradient_policy=None)
    a.device = torch.device("cpu")  # use_cuda=False
    with pytest.raises(ValueError, match="GPU only"):
        a.init_model()
