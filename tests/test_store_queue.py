"""State store (LocalStore and the TCP server/client pair), task queue semantics and the
worker planning policies."""
import threading
import time

import pytest

from thinvids_amd.store import LocalStore, RemoteStore
from thinvids_amd.store.server import StoreServer


@pytest.fixture(params=["local", "tcp"])
def store(request):
    if request.param == "local":
        yield LocalStore()
        return
    srv = StoreServer("127.0.0.1", 0)
    srv.start_background()
    yield RemoteStore("127.0.0.1", srv.server_address[1], retries=1)
    srv.shutdown()
    srv.server_close()


def test_store_types_and_expiry(store):
    assert store.set("k", "v") and store.get("k") == "v"
    assert store.set("k", "w", nx=True) in (None, False) and store.get("k") == "v"
    assert store.incr("n") == 1 and store.incrby("n", 5) == 6
    store.hset("h", mapping={"a": 1, "b": "x"})
    assert store.hgetall("h") == {"a": "1", "b": "x"} and store.hincrby("h", "a", 2) == 3
    assert store.hmget("h", ["a", "zz"]) == ["3", None]
    assert store.sadd("s", "x", "y") == 2 and store.sismember("s", "x") and store.scard("s") == 2
    assert store.smembers("s") == {"x", "y"}
    store.rpush("l", "1", "2", "3")
    assert store.lrange("l", 0, -1) == ["1", "2", "3"] and store.lpop("l") == "1"
    store.ltrim("l", 0, 0)
    assert store.lrange("l", 0, -1) == ["2"]
    store.set("t", "1", ex=1)
    assert 0 < store.ttl("t") <= 1
    time.sleep(1.1)
    assert store.get("t") is None
    assert sorted(store.keys("h*")) == ["h"]
    p = store.pipeline()
    p.hget("h", "b")
    p.scard("s")
    assert p.execute() == ["x", 2]
    assert store.delete("h", "s") == 2 and not store.exists("h")


def test_blpop_wakes_on_push(store):
    got = []

    def waiter():
        got.append(store.blpop(["q"], timeout=5))

    t = threading.Thread(target=waiter)
    t.start()
    time.sleep(0.2)
    store.rpush("q", "hello")
    t.join(5)
    assert got == [("q", "hello")] or got == [["q", "hello"]]
    assert store.blpop(["q"], timeout=0.1) is None


def test_wrong_type(store):
    store.set("x", "1")
    with pytest.raises(Exception):
        store.hset("x", "f", "v")


def test_queue_retry_revoke_and_batch():
    from thinvids_amd.queue import TaskQueue

    st = LocalStore()
    q = TaskQueue("unit", store=st)
    calls = []

    @q.task(retries=2)
    def flaky(x):
        calls.append(x)
        if len(calls) < 3:
            raise RuntimeError("boom")
        return x

    flaky(7)
    assert q.drain() == 3 and calls == [7, 7, 7]
    tid = flaky(8)
    q.revoke_by_id(tid)
    assert q.drain() == 0 and len(q) == 0 and calls[-1] == 7  # revoked task is dropped

    @q.task()
    def enc(job, idx):
        return idx

    for i in range(5):
        enc("a" if i % 2 == 0 else "b", i)
    batch = q.pop_batch(8, lambda a, b: a["args"][0] == b["args"][0])
    assert [m["args"][1] for m in batch] == [0, 2, 4]
    assert [m["args"][1] for m in q.pending()] == [1, 3]
    delayed = q.enqueue("enc", ["a", 9], delay=30)
    assert q.pop(timeout=0.05) is not None  # message 1 is due
    assert any(m["id"] == delayed for m in q.pending())


def test_plan_parts_policy():
    from thinvids_amd.worker.planning import plan_parts

    p = plan_parts(1000, usable_encoders=8, gop=64)
    assert p.effective_parts % 8 == 0 and sum(n for _, _, n in p.ranges) == 1000
    assert p.ranges[0][0] == 1 and p.ranges[1][1] == p.frames_per_part
    p = plan_parts(1000, usable_encoders=3, gop=64, segment_frames=100)
    assert p.requested_parts == 10 and p.effective_parts == 12
    assert plan_parts(0, 4).ranges == []
    assert plan_parts(20, 16, gop=4, min_frames=8).effective_parts == 2  # never tiny parts


def test_redispatch_policy():
    from thinvids_amd.worker.planning import StitchTunables, plan_redispatch

    t = StitchTunables(max_retries=2, retry_interval_sec=10, stall_before_retry_sec=30, miss_min_age_sec=20,
                       retry_window_ahead=4, max_parallel_redispatch=2)
    now = 1000.0
    newly, retry, give = plan_redispatch({1, 2, 5}, 10, 10, now, now - 5, {}, {}, {}, 10, t)
    assert newly == [3, 4, 6] and retry == [] and not give  # not stalled yet
    seen = {3: now - 100, 4: now - 100, 6: now - 5}
    newly, retry, give = plan_redispatch({1, 2, 5}, 10, 10, now, now - 60, seen, {}, {}, 10, t)
    assert newly == [] and retry == [3, 4] and not give  # oldest misses, capped at 2
    newly, retry, give = plan_redispatch({1, 2, 5}, 10, 10, now, now - 60, seen, {3: 2}, {3: now - 100}, 10, t)
    assert 3 not in retry and give  # retry budget exhausted long ago -> give up


def test_batch_refuses_private_nested_and_blocking_ops():
    import json
    import socket

    srv = StoreServer("127.0.0.1", 0)
    srv.start_background()
    try:
        srv.store.set("keep", "1")
        s = socket.create_connection(srv.server_address)
        f = s.makefile("rwb")
        for bad in (["__init__", [], {}], ["blpop", [["q"], 0], {}], ["execute_batch", [[]], {}],
                    ["_new", ["x", "string"], {}]):
            f.write((json.dumps({"batch": [["set", ["a", "1"], {}], bad]}) + "\n").encode())
            f.flush()
            resp = json.loads(f.readline())
            assert "err" in resp and "not allowed" in resp["err"], resp
        f.write((json.dumps({"op": "__init__", "args": []}) + "\n").encode())
        f.flush()
        assert "err" in json.loads(f.readline())
        assert srv.store.get("keep") == "1" and srv.store.get("a") is None  # nothing ran
        with pytest.raises(ValueError):
            LocalStore().execute_batch([("blpop", [["q"], 0], {})])
        s.close()
    finally:
        srv.shutdown()
        srv.server_close()
