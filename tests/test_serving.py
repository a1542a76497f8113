"""Cluster Serving (ClusterServingSpec / PreProcessingSpec / PostProcessingSpec /
test_serving client analogues): the RESP queue server, the end-to-end
enqueue -> batch -> infer -> result path, pre/post processing formats."""
import numpy as np
import pytest
import torch

from zoo.common.nncontext import init_nncontext


@pytest.fixture(scope="module", autouse=True)
def ctx():
    return init_nncontext()


@pytest.fixture(params=["native", "python"])
def server(request):
    from zoo.serving.resp import NativeRespServer, PyRespServer
    cls = NativeRespServer if request.param == "native" else PyRespServer
    srv = cls("127.0.0.1", 0, maxmemory=1 << 20).start()
    yield srv
    srv.shutdown()
    srv.server_close()


def test_resp_streams_hashes_groups(server):
    from zoo.serving.resp import RespClient
    c = RespClient("127.0.0.1", server.port)
    assert c.ping()
    c.xgroup_create("s", "g", id="0", mkstream=True)
    ids = [c.xadd("s", {"uri": "u%d" % i, "v": str(i)}) for i in range(5)]
    assert c.xlen("s") == 5
    got = c.xreadgroup("g", "c1", {"s": ">"}, count=3, block=10)
    msgs = got[0][1]
    assert [m[1][b"uri"] for m in msgs] == [b"u0", b"u1", b"u2"]
    got2 = c.xreadgroup("g", "c2", {"s": ">"}, count=10, block=10)
    assert [m[1][b"uri"] for m in got2[0][1]] == [b"u3", b"u4"]  # consumer group: no re-delivery
    assert c.xreadgroup("g", "c1", {"s": ">"}, count=1, block=20) == []
    assert c.xack("s", "g", *ids) == 5 and c.xdel("s", *ids) == 5 and c.xlen("s") == 0
    c.hset("result:a", "value", "[1,2]")
    assert c.hgetall("result:a") == {b"value": b"[1,2]"}
    assert c.keys("result:*") == [b"result:a"]
    assert c.delete("result:a") == 1 and c.exists("result:a") == 0
    info = c.info()
    assert info["maxmemory"] == 1 << 20
    # back-pressure: the server refuses writes beyond maxmemory
    with pytest.raises(Exception):
        for i in range(10000):
            c.xadd("big", {"x": "y" * 4096})


def test_post_processing_formats():
    from zoo.serving.server import post_process
    t = np.array([0.1, 0.7, 0.2], np.float32)
    assert post_process(t, "topN(2)") == "[[1,%r][2,%r]]" % (float(np.float32(0.7)), float(np.float32(0.2)))
    s = post_process(np.array([[1.0, 2.0], [3.0, 4.0]], np.float32))
    assert s == "[[1.0,2.0],[3.0,4.0]]"
    with pytest.raises(ValueError):
        post_process(t, "topN(2")


def test_serving_end_to_end_tensors_and_images(server, tmp_path):
    from zoo.serving import ClusterServing, InputQueue, OutputQueue
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Flatten(), torch.nn.Linear(3 * 8 * 8, 5), torch.nn.Softmax(-1))
    cfg = tmp_path / "config.yaml"
    cfg.write_text("model:\n  path: m\ndata:\n  src: 127.0.0.1:%d\n  image_shape: 3,8,8\n  filter: topN(2)\n"
                   "params:\n  batch_size: 4\n" % server.port)
    serving = ClusterServing(str(cfg), model=model)
    inq, outq = InputQueue(str(cfg)), OutputQueue(str(cfg))
    rng = np.random.default_rng(0)
    xs = {("t%d" % i): rng.random((3, 8, 8)).astype(np.float32) for i in range(6)}
    for k, v in xs.items():
        inq.enqueue_tensor(k, v)
    img = rng.integers(0, 255, (10, 12, 3)).astype(np.uint8)
    inq.enqueue_image("img0", img)
    served = serving.run(max_records=7, idle_timeout=5)
    assert served == 7
    res = outq.dequeue()
    assert set(res) == set(xs) | {"img0"}
    import copy
    with torch.no_grad():   # (serving moved the model to its device; the reference runs on the CPU)
        ref = copy.deepcopy(model).cpu()(torch.from_numpy(xs["t3"][None]))[0].numpy()
    top = np.argsort(-ref)[:2]
    assert res["t3"].startswith("[[%d," % top[0]) and ("[%d," % top[1]) in res["t3"]
    assert outq.dequeue() == {}


def test_model_discovery(tmp_path):
    from zoo.serving.server import discover_model
    (tmp_path / "a.prototxt").write_text("x")
    (tmp_path / "a.caffemodel").write_bytes(b"")
    kind, files = discover_model(str(tmp_path))
    assert kind == "caffe" and len(files) == 2
    (tmp_path / "m.onnx").write_bytes(b"")
    assert discover_model(str(tmp_path / "m.onnx"))[0] == "onnx"


def test_native_store_commands_and_concurrency(server):
    """Both servers agree on XRANGE/KEYS globbing/DEL/FLUSHALL, and many concurrent
    producers plus a blocking consumer group lose and duplicate nothing."""
    import threading
    from zoo.serving.resp import RespClient
    c = RespClient("127.0.0.1", server.port)
    c.xgroup_create("s", "g", id="0", mkstream=True)
    ids = [c.xadd("s", {"k": str(i)}) for i in range(4)]
    rng = c.execute_command("XRANGE", "s", "-", "+", "COUNT", 3)
    assert [r[0] for r in rng] == ids[:3]
    for k in ("result:a1", "result:b2", "other"):
        c.hset(k, "value", "x")
    assert sorted(c.keys("result:[a-b]?")) == [b"result:a1", b"result:b2"]
    assert c.execute_command("DBSIZE") == 4
    assert c.execute_command("FLUSHALL") in ("OK", b"OK")
    assert c.keys("*") == []
    c.xgroup_create("q", "g", id="0", mkstream=True)
    n_prod, per = 4, 50

    def prod(p):
        cc = RespClient("127.0.0.1", server.port)
        for i in range(per):
            cc.xadd("q", {"uri": "p%d-%d" % (p, i)})
    ths = [threading.Thread(target=prod, args=(p,)) for p in range(n_prod)]
    for t in ths:
        t.start()
    seen = []
    while len(seen) < n_prod * per:
        got = c.xreadgroup("g", "w", {"q": ">"}, count=16, block=200)
        for _, msgs in got:
            seen += [m[1][b"uri"] for m in msgs]
    for t in ths:
        t.join()
    assert len(seen) == len(set(seen)) == n_prod * per


def test_native_local_client_fast_paths():
    from zoo.serving.resp import NativeRespServer, RespClient, connect
    import base64
    srv = NativeRespServer("127.0.0.1", 0, 1 << 20)
    try:
        lc = connect("127.0.0.1", srv.port, local=True)
        assert type(lc).__name__ == "LocalClient"
        lc.xgroup_create("image_stream", "serving", id="0", mkstream=True)
        rc = RespClient("127.0.0.1", srv.port)
        rc.xadd("image_stream", {"uri": "a", "image": base64.b64encode(b"\x01\x02jpeg")})
        rc.xadd("image_stream", {"uri": "b", "tensor": base64.b64encode(np.ones(3, np.float32).tobytes()),
                                 "shape": "3"})
        recs = lc.read_batch("image_stream", "serving", "w", 8, 50)
        assert [(r[1], r[2]) for r in recs] == [("a", "image"), ("b", "tensor")]
        assert recs[0][3] == b"\x01\x02jpeg" and np.frombuffer(recs[1][3], np.float32).tolist() == [1.0] * 3
        lc.finish("image_stream", "serving", [r[0] for r in recs], [("result:a", "[1]"), ("result:b", "[2]")])
        assert rc.xlen("image_stream") == 0 and rc.hgetall("result:b") == {b"value": b"[2]"}
        assert lc.read_batch("image_stream", "serving", "w", 8, 10) == []
    finally:
        srv.shutdown()


def test_post_process_batch_matches_per_row_top_n():
    """the vectorised topN post-processing (worker hot path) is string-identical to the
    per-row PostProcessing.topN, ties included"""
    import numpy as np
    from zoo.serving.server import post_process, post_process_batch
    rng = np.random.default_rng(0)
    for F in (3, 10, 768, 1000):
        a = rng.standard_normal((32, F)).astype(np.float32)
        a[3, :] = 0.5
        a[4, :7] = 2.0
        a[5] = np.round(a[5])
        for n in (1, 5):
            flt = "topN(%d)" % n
            assert post_process_batch(a, flt) == [post_process(r, flt) for r in a]
    b = rng.standard_normal((4, 6)).astype(np.float32)
    assert post_process_batch(b, "None") == [post_process(r, "None") for r in b]


@pytest.mark.parametrize("tcp", [False, True])
def test_native_open_loop_load_generator(tcp):
    """The C++ open-loop generator (csrc/runtime/serving.cpp run_loadgen) against a store with a
    consumer that answers in batches: every record sent on schedule, latencies from the store's
    finish stamps, achieved ~= offered below capacity; over TCP it goes through the RESP server."""
    import base64
    import threading
    import time
    from zoo import _runtime
    st = _runtime.NativeStore(1 << 28)
    st.serve("127.0.0.1", 0)
    try:
        st.execute([b"XGROUP", b"CREATE", b"image_stream", b"serving", b"0", b"MKSTREAM"])
        st.track(True)
        stop = threading.Event()

        def consumer():
            while not stop.is_set():
                recs = st.read_batch("image_stream", "serving", "c0", 32, 10)
                if recs:
                    time.sleep(0.001)
                    st.finish("image_stream", "serving", [r[0].decode() for r in recs],
                              [("result:" + r[1], "ok") for r in recs], "value")

        th = threading.Thread(target=consumer, daemon=True)
        th.start()
        payloads = [base64.b64encode(bytes([i]) * 500).decode() for i in range(4)]
        d = st.loadgen("image_stream", "image", payloads, "", 2000.0, 1.5, 3, "t", 0.5, 5.0, tcp)
        stop.set()
        th.join(5)
        assert d["sent"] == 3000 and d["unfinished"] == 0
        assert d["measured"] == d["completed"] > 1500
        assert abs(d["offered_rate"] - 2000.0) < 1.0
        assert 1700 < d["achieved_throughput"] < 2300
        assert 0 < d["p50_ms"] <= d["p90_ms"] <= d["p99_ms"] <= d["max_ms"] < 1000
        # the records carry the uri / payload a worker decodes
        assert st.execute([b"EXISTS", b"result:t-0"]) == 1
    finally:
        st.stop()


def test_native_store_growth_has_no_stop_the_world_rehash():
    """Result keys spread over 64 hash tables (csrc/runtime/serving.cpp ShardedMap): writing 300k
    results never stalls one finish() call for a whole-table rehash (the r6 serving tail, a 20-40
    ms stop every time the single table doubled); the keyspace commands see every shard."""
    import time
    from zoo import _runtime
    st = _runtime.NativeStore(1 << 30)
    st.track(True)
    worst, n, b = 0.0, 4688 * 64, 64
    for i in range(0, n, b):
        res = [("result:g-%d" % j, "v") for j in range(i, i + b)]
        t = time.perf_counter()
        st.finish("image_stream", "serving", [], res, "value")
        worst = max(worst, time.perf_counter() - t)
    assert st.execute([b"DBSIZE"]) == n
    assert worst < 0.012, worst   # the single-table store: 88-99 ms worst call here
    keys = st.execute([b"KEYS", b"result:g-29999?"])
    assert sorted(keys) == sorted(("result:g-29999%d" % d).encode() for d in range(10))
    assert st.execute([b"DEL", b"result:g-0", b"result:g-1", b"nope"]) == 2
    assert st.execute([b"EXISTS", b"result:g-0", b"result:g-2"]) == 1
    assert st.execute([b"HGET", b"result:g-2", b"value"]) == b"v"
    st.execute([b"FLUSHALL"])
    assert st.execute([b"DBSIZE"]) == 0
