"""Zero-copy payload ingress (fedscale_amd/ingress.py + fa_pickle_strip): ``ingress.loads`` must return
what ``pickle.loads`` returns (aggregator.py:704) for every payload the executor can send
(torch_client.py:76-91), and fall back to ``pickle.loads`` for anything else.  Host-only code: runs on CPU."""
import ctypes
import pickle

import numpy as np
import pytest

from fedscale_amd import _native, ingress


@pytest.fixture(autouse=True)
def _fast_path_for_small_payloads(monkeypatch):
    """The cases here are small; exercise the zero-copy path on them (production: >= MIN_PAYLOAD)."""
    monkeypatch.setattr(ingress, "MIN_PAYLOAD", 0)


def _assert_same(a, b, path="root"):
    assert type(a) is type(b), path
    if isinstance(a, np.ndarray):
        assert a.dtype == b.dtype and a.shape == b.shape, path
        assert a.flags.f_contiguous == b.flags.f_contiguous and a.flags.c_contiguous == b.flags.c_contiguous
        assert a.tobytes() == b.tobytes(), path  # bitwise (NaN payloads included)
    elif isinstance(a, dict):
        assert list(a.keys()) == list(b.keys()), path
        for k in a:
            _assert_same(a[k], b[k], f"{path}.{k}")
    elif isinstance(a, (list, tuple)):
        assert len(a) == len(b), path
        for i, (x, y) in enumerate(zip(a, b)):
            _assert_same(x, y, f"{path}[{i}]")
    else:
        assert a == b or (a != a and b != b), path


def _executor_result(seed=0, scale=1):
    """Shape of torch_client.py:76-91's result for a small ResNet-like state_dict."""
    rng = np.random.default_rng(seed)
    w = {}
    for i in range(6):
        w[f"layer{i}.conv.weight"] = rng.standard_normal((16 * scale, 8, 3, 3), dtype=np.float32)
        w[f"layer{i}.bn.weight"] = rng.standard_normal(16 * scale, dtype=np.float32)
        w[f"layer{i}.bn.running_var"] = rng.random(16 * scale, dtype=np.float32)
        w[f"layer{i}.bn.num_batches_tracked"] = np.array(7 + i, dtype=np.int64)
    w["fc.weight"] = rng.standard_normal((10, 512 * scale), dtype=np.float32)
    w["fc.weight"][0, :4] = [np.nan, np.inf, -np.inf, -0.0]
    return {"client_id": 3 + seed, "moving_loss": 1.25, "trained_size": 200, "success": True,
            "utility": 17.5, "update_weight": w, "wall_duration": 0}


def test_executor_result_roundtrip():
    r = _executor_result()
    b = pickle.dumps(r)
    got = ingress.loads(b)
    _assert_same(got, pickle.loads(b))
    # large arrays really are views of the payload (no copy), small ones are rebuilt inline
    big = got["update_weight"]["layer0.conv.weight"]
    assert not big.flags.writeable and big.base is not None
    assert got["update_weight"]["layer0.bn.num_batches_tracked"].flags.writeable


def test_strip_regions_point_at_array_bytes():
    r = _executor_result(seed=1)
    b = pickle.dumps(r)
    stream, regions = ingress.strip(b, ingress.MIN_BYTES)
    big = [a for a in r["update_weight"].values() if a.nbytes >= ingress.MIN_BYTES]
    assert len(regions) == len(big)
    for a, (off, n) in zip(big, regions):
        assert n == a.nbytes and b[off:off + n] == a.tobytes()
    assert len(stream) < len(b) - sum(a.nbytes for a in big) + 14 * len(big)


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.float16, np.int64, np.int32, np.uint8, np.bool_,
                                   np.complex64])
def test_dtypes_and_layouts(dtype):
    rng = np.random.default_rng(2)
    base = (rng.standard_normal((70, 90)) * 50)
    a = base.astype(dtype) if dtype is not np.complex64 else (base + 1j * base).astype(dtype)
    obj = {"c": np.ascontiguousarray(a), "f": np.asfortranarray(a), "t": a.T, "s": a[::2, 1:],
           "e": np.empty((0, 5000), dtype), "z": np.zeros((64, 64), dtype)}
    b = pickle.dumps(obj)
    _assert_same(ingress.loads(b, min_bytes=64), pickle.loads(b))


def test_nested_containers_and_shared_arrays():
    a = np.arange(20000, dtype=np.float32)
    obj = {"l": [a, (a, 1.0), {"x": a}], "t": (np.ones(5000, np.int64), "s"), "k": [[np.zeros(3000)]]}
    b = pickle.dumps(obj)
    got = ingress.loads(b)
    _assert_same(got, pickle.loads(b))
    # memoised once in the pickle -> one object after loading, as with pickle.loads
    assert got["l"][0] is got["l"][1][0] is got["l"][2]["x"]


@pytest.mark.parametrize("case", ["bytes_blob", "object_array", "subclass", "custom_object", "protocol2",
                                  "protocol5", "small", "bytearray"])
def test_fallback_cases_match_pickle(case):
    big = np.arange(10000, dtype=np.float32)
    if case == "bytes_blob":
        obj = {"w": big, "blob": b"\x01" * 10000}
    elif case == "object_array":
        obj = {"w": big, "o": np.array([{"a": 1}, "x", 3.0] * 2000, dtype=object)}
    elif case == "subclass":
        obj = {"w": big, "m": np.ma.masked_array(big, mask=big > 5000)}
    elif case == "custom_object":
        import collections

        obj = {"w": collections.OrderedDict(a=big)}
    elif case == "small":
        obj = {"w": np.arange(10, dtype=np.float32)}
    elif case == "bytearray":
        obj = {"w": big, "b": bytearray(b"\x02" * 9000)}
    else:
        obj = {"w": big, "n": 3}
    proto = {"protocol2": 2, "protocol5": 5}.get(case, 4)
    b = pickle.dumps(obj, protocol=proto)
    got, ref = ingress.loads(b), pickle.loads(b)
    assert type(got) is type(ref) and list(got) == list(ref)
    assert pickle.dumps(got, protocol=4) == pickle.dumps(ref, protocol=4)


def test_truncated_payload_raises_like_pickle():
    b = pickle.dumps(_executor_result())
    for cut in (len(b) // 2, len(b) - 1):
        with pytest.raises(Exception) as ref:
            pickle.loads(b[:cut])
        with pytest.raises(type(ref.value)):
            ingress.loads(b[:cut])


def test_strip_error_paths():
    lib = _native.load()
    n = ctypes.c_int32(0)
    regions = (ctypes.c_int64 * 8)()
    good = pickle.dumps({"w": np.ones(5000, np.float32)})
    assert lib.fa_pickle_strip(good, len(good), 8, None, 0, regions, 4, ctypes.byref(n)) < 0   # min_bytes < 16
    assert lib.fa_pickle_strip(good, len(good) - 1, 64, None, 0, regions, 4, ctypes.byref(n)) < 0  # no STOP
    p5 = pickle.dumps(pickle.PickleBuffer(np.ones(100, np.uint8)), protocol=5, buffer_callback=lambda _: False)
    assert lib.fa_pickle_strip(p5, len(p5), 64, None, 0, regions, 4, ctypes.byref(n)) < 0  # out-of-band
    # sizing call (out=NULL) reports the exact stripped length; the second call fills it
    need = lib.fa_pickle_strip(good, len(good), 64, None, 0, regions, 4, ctypes.byref(n))
    assert need > 0 and n.value == 1
    out = ctypes.create_string_buffer(need)
    assert lib.fa_pickle_strip(good, len(good), 64, out, need, regions, 4, ctypes.byref(n)) == need
    assert out.raw.count(b"FAPB") == 1 and regions[1] == 20000


def test_aggregator_deserialize_hook():
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregatorMixin

    class Base:
        def deserialize_response(self, responses):
            return ("converted", pickle.loads(responses))

    class Plain(DeviceAggregatorMixin):
        pass

    class Converting(DeviceAggregatorMixin, Base):
        pass

    b = pickle.dumps(_executor_result(scale=4))
    got = Plain().deserialize_response(b)
    _assert_same(got, pickle.loads(b))
    assert not got["update_weight"]["fc.weight"].flags.writeable
    # a base class that converts the payload keeps its own path
    assert Converting().deserialize_response(b)[0] == "converted"
    off = Plain()
    off.device_zero_copy_ingress = False
    assert off.deserialize_response(b)["update_weight"]["fc.weight"].flags.writeable


def test_egress_handle_and_mixin_guards():
    """EgressHandle (host-only part) and the mixin's guards: a plugin's own create_client_task /
    get_test_config (async_aggregator.py:40, examples/auxo/aggregator.py:156,254) are left alone."""
    import torch

    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregatorMixin
    from fedscale_amd.cloud.internal.torch_model_adapter import EgressHandle

    ws = [torch.arange(6, dtype=torch.float32).reshape(2, 3), torch.tensor(4, dtype=torch.int64)]
    payload = pickle.dumps(ws)
    h = EgressHandle((1, 2), payload)
    assert h._weights is None  # nothing unpickled until the handle is used as a list
    assert len(h) == 2 and torch.equal(h[0], ws[0]) and torch.equal(list(h)[1], ws[1])
    assert type(pickle.loads(pickle.dumps(h))) is list

    class Plain(DeviceAggregatorMixin):
        pass

    assert Plain().serialize_response(h) is payload

    class AsyncAggregator:  # a plugin with its own create_client_task
        def create_client_task(self, executor_id):
            return "plugin", executor_id

        def get_test_config(self, client_id):
            return "plugin-test", client_id

    class Wrapped(DeviceAggregatorMixin, AsyncAggregator):
        pass

    assert Wrapped().create_client_task(7) == ("plugin", 7)
    assert Wrapped().get_test_config(8) == ("plugin-test", 8)


def test_egress_bytes_of_past_versions_cached_per_list():
    """FedBuff's create_client_task hands out the model_cache lists of past versions
    (async_aggregator.py:54): each list object is pickled once, and the bytes are pickle.dumps of it."""
    import torch

    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregatorMixin
    from fedscale_amd.cloud.internal.torch_model_adapter import EgressWeights

    class Plain(DeviceAggregatorMixin):
        model_wrapper = None

    agg = Plain()
    lists = []
    for v in range(10):
        w = EgressWeights([torch.full((3, 2), float(v)), torch.tensor(v, dtype=torch.int64)])
        w.egress_key = (12345, v)  # no adapter of this aggregator holds these versions
        lists.append(w)
    b0 = agg.serialize_response(lists[0])
    assert agg.serialize_response(lists[0]) is b0
    assert b0 == pickle.dumps([lists[0][0], lists[0][1]])
    assert type(pickle.loads(b0)) is list
    for w in lists[1:]:
        agg.serialize_response(w)
    assert len(agg._egress_past) == agg.device_egress_past_versions
    b0_again = agg.serialize_response(lists[0])  # evicted: pickled again, same bytes
    assert b0_again == b0 and b0_again is not b0


def test_torch_state_dict_payload_falls_back():
    """HeteroFL clients upload a torch state_dict (examples/heterofl/customized_client.py:93): tensors
    pickle through torch's own reducers, which the fast path does not rebuild; the result is still
    exactly pickle.loads'."""
    from collections import OrderedDict

    import torch

    sd = OrderedDict(w=torch.arange(5000, dtype=torch.float32).reshape(50, 100), n=torch.tensor(3))
    b = pickle.dumps({"client_id": 1, "local_parameters": sd, "update_weight": {"x": np.ones(4096, np.float32)}})
    got, ref = ingress.loads(b), pickle.loads(b)
    assert type(got["local_parameters"]) is OrderedDict
    for k in sd:
        assert torch.equal(got["local_parameters"][k], ref["local_parameters"][k])
    assert np.array_equal(got["update_weight"]["x"], ref["update_weight"]["x"])


def test_small_payloads_take_pickle_loads(monkeypatch):
    """Below MIN_PAYLOAD the fast path costs more than pickle's copy: plain pickle.loads (writable arrays)."""
    monkeypatch.setattr(ingress, "MIN_PAYLOAD", 1 << 20)
    b = pickle.dumps(_executor_result())
    assert len(b) < 1 << 20
    got = ingress.loads(b)
    assert got["update_weight"]["fc.weight"].flags.writeable
    _assert_same(got, pickle.loads(b))
    big = pickle.dumps(_executor_result(scale=64))
    assert len(big) >= 1 << 20
    assert not ingress.loads(big)["update_weight"]["fc.weight"].flags.writeable


def test_client_ping_update_model_hands_out_the_egress_handle():
    """The reference servicer's UPDATE_MODEL branch (aggregator.py:902-907) serialises
    model_wrapper.get_weights(): under the mixin that one call returns the adapter's EgressHandle (no
    clone); other events, other threads, the opt-out and a plugin's own CLIENT_PING keep get_weights()."""
    import collections
    import threading
    import types

    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregatorMixin
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    class FakeAdapter(TorchModelAdapter):  # only the egress part of the adapter
        def __init__(self):
            self.clones = 0

        def egress_handle(self):
            return "HANDLE"

        def _preallocate_clones(self):
            return None

        def _acquire_host(self):
            self.clones += 1
            raise LookupError("clone path")

    class Aggregator:  # the shape of the reference CLIENT_PING (aggregator.py:870-912)
        def CLIENT_PING(self, request, context):
            ev = self.individual_client_events[request.executor_id].popleft()
            if ev == "update_model":
                try:
                    data = self.model_wrapper.get_weights()
                except LookupError:
                    data = "CLONE"
                # a second call in the same ping is not covered by the one-shot
                try:
                    self.model_wrapper.get_weights()
                except LookupError:
                    pass
                return ev, data
            return ev, None

    class Agg(DeviceAggregatorMixin, Aggregator):
        pass

    agg = Agg()
    agg.model_wrapper = FakeAdapter()
    agg.individual_client_events = {1: collections.deque(["update_model", "model_test", "update_model"])}
    req = types.SimpleNamespace(executor_id=1, client_id=1)
    assert agg.CLIENT_PING(req, None) == ("update_model", "HANDLE")
    assert agg.model_wrapper.clones == 1  # the second get_weights() cloned
    assert agg.CLIENT_PING(req, None) == ("model_test", None)
    out = []
    t = threading.Thread(target=lambda: out.append(agg.CLIENT_PING(req, None)))
    t.start()
    t.join()
    assert out == [("update_model", "HANDLE")]
    # the flag does not leak out of the ping
    try:
        agg.model_wrapper.get_weights()
    except LookupError:
        pass
    assert agg.model_wrapper.clones == 3
    agg.device_egress_handles = False
    agg.individual_client_events[1].append("update_model")
    assert agg.CLIENT_PING(req, None) == ("update_model", "CLONE")

    class PluginPing:
        def CLIENT_PING(self, request, context):
            return "plugin", None

    class Wrapped(DeviceAggregatorMixin, PluginPing):
        pass

    w = Wrapped()
    w.model_wrapper = FakeAdapter()
    w.individual_client_events = {1: collections.deque(["update_model"])}
    assert w.CLIENT_PING(req, None) == ("plugin", None)
    assert w.individual_client_events[1] == collections.deque(["update_model"])


def test_upload_decoded_on_arrival_by_the_servicer_thread():
    """add_event_handler (aggregator.py:830-840) runs on the servicer thread: an UPLOAD_MODEL payload is
    decoded there and the main loop's deserialize_response (:993-994) hands the result back; other events,
    undecodable payloads, the opt-out and a plugin's own deserialize_response keep the raw bytes."""
    import collections
    import threading

    import numpy as np

    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregatorMixin

    class Aggregator:  # the reference methods the mixin wraps
        def __init__(self):
            self.server_events_queue = collections.deque()

        def add_event_handler(self, client_id, event, meta, data):
            self.server_events_queue.append((client_id, event, meta, data))

        def deserialize_response(self, responses):
            return pickle.loads(responses)

    class Agg(DeviceAggregatorMixin, Aggregator):
        pass

    rng = np.random.default_rng(3)
    upd = {"w": rng.standard_normal((512, 1024), dtype=np.float32), "n": np.array(7, dtype=np.int64)}
    res = {"client_id": 4, "update_weight": upd, "moving_loss": 0.5}
    payload = pickle.dumps(res, protocol=4)
    agg = Agg()
    agg.add_event_handler(9, "upload_model", None, payload)  # off by default: the reference's queue entry
    assert agg.server_events_queue.popleft()[3] is payload
    agg.device_decode_on_arrival = True
    t = threading.Thread(target=agg.add_event_handler, args=(4, "upload_model", "meta", payload))
    t.start()
    t.join()
    agg.add_event_handler(4, "model_test", "meta", pickle.dumps({"acc": 1.0}))
    agg.add_event_handler(5, "upload_model", "meta", payload[:-9])  # truncated: queued as it came
    (c, ev, meta, data), (_, ev2, _, data2), (_, _, _, data3) = agg.server_events_queue
    assert (c, ev, meta) == (4, "upload_model", "meta") and type(data) is not bytes
    got = agg.deserialize_response(data)
    assert got["client_id"] == 4 and np.array_equal(got["update_weight"]["w"], upd["w"])
    assert got["update_weight"]["n"] == 7
    assert type(data2) is bytes and agg.deserialize_response(data2) == {"acc": 1.0}
    assert data3 == payload[:-9]
    with pytest.raises(Exception):
        agg.deserialize_response(data3)
    agg.device_decode_on_arrival = False
    agg.add_event_handler(6, "upload_model", None, payload)
    assert agg.server_events_queue[-1][3] is payload

    class Converting(Aggregator):  # e.g. aggregator_tflite.py:47-58
        def deserialize_response(self, responses):
            return ("converted", pickle.loads(responses)["client_id"])

    class Wrapped(DeviceAggregatorMixin, Converting):
        pass

    w = Wrapped()
    w.device_decode_on_arrival = True
    w.add_event_handler(1, "upload_model", None, payload)
    assert w.server_events_queue[0][3] is payload and w.deserialize_response(payload) == ("converted", 4)

    class Standalone(DeviceAggregatorMixin):
        pass

    s = Standalone()
    s.device_decode_on_arrival = True
    s.add_event_handler(1, "upload_model", None, payload)
    assert s.deserialize_response(s.server_events_queue[0][3])["client_id"] == 4


def test_sharded_registration_reuse_checks_the_end_page(monkeypatch):
    """an upload whose first payload page an EARLIER registration already covers may reuse that
    registration only if it ends inside it; a payload that extends past it takes the pinned-row gather (counted in
    ``registration_fallbacks``) instead of reaching fa_h2d_pieces with unregistered tail pages.  CPU: the adapter's
    registration bookkeeping alone, the native calls recorded."""
    import torch

    from fedscale_amd import synth
    from fedscale_amd.bucket import BucketLayout
    from fedscale_amd.cloud.internal.sharded_model_adapter import ShardedModelAdapter

    names, shapes = ["a.weight", "b.weight"], [(512, 1024), (512, 1024)]
    model = synth.LayoutModule(names, shapes, [torch.float32] * 2)
    L = BucketLayout.from_state_dict(model.state_dict())
    rng = np.random.default_rng(0)
    up = {n: rng.standard_normal(s, dtype=np.float32) for n, s in zip(names, shapes)}
    payload = pickle.dumps({"update_weight": up})
    dec = ingress.loads(payload)["update_weight"]
    calls = []
    monkeypatch.setattr(_native, "call", lambda name, *a: calls.append((name,) + a) or 0)

    class _Pending:  # a registration whose copies are still running
        events = [type("E", (), {"query": staticmethod(lambda: False)})()]

    ad = ShardedModelAdapter.__new__(ShardedModelAdapter)
    ad.layout, ad._reg_segs, ad._regs = L, None, {}
    ad.registered_uploads = ad.registration_fallbacks = 0
    plan = L.host_gather_plan(L.values_of(dec))
    buf = np.frombuffer(payload, dtype=np.uint8)
    a0 = buf.ctypes.data // 4096 * 4096
    a1 = -(-(buf.ctypes.data + buf.nbytes) // 4096) * 4096
    # an earlier payload's registration starting on the same page but ending one page short of this one
    ad._regs[a0] = [b"earlier", [_Pending()], a1 - 4096]
    assert ad._register(plan) is None
    assert ad.registration_fallbacks == 1 and not any(c[0] == "fa_host_register" for c in calls)
    # one that covers the whole payload is reused (no second registration)
    ad._regs[a0] = [b"earlier", [_Pending()], a1]
    got = ad._register(plan)
    assert got is not None and got[2] == a0 and ad.registration_fallbacks == 1
    assert not any(c[0] == "fa_host_register" for c in calls)
