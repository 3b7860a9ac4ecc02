"""Tracing spans (ROCTx + Chrome trace export) and misc utilities."""
import json
import os
import threading

import pytest


def test_trace_spans_summary_and_chrome_export(tmp_path, monkeypatch):
    from thinvids_amd.utils import trace

    monkeypatch.setenv("TV_TRACE_FILE", str(tmp_path / "t.json"))
    trace.summary(reset=True)

    def work():
        for _ in range(3):
            with trace.span("stage.a", k=1):
                pass

    ts = [threading.Thread(target=work) for _ in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    with trace.span("stage.b"):
        trace.mark("m")
    s = trace.summary()
    assert s["stage.a"]["count"] == 6 and s["stage.b"]["count"] == 1
    assert s["stage.a"]["max_ms"] >= s["stage.a"]["avg_ms"] >= 0
    path = trace.flush()
    ev = json.load(open(path))["traceEvents"]
    assert sum(e["name"] == "stage.a" and e["ph"] == "X" for e in ev) >= 6
    assert any(e["ph"] == "i" and e["name"] == "m" for e in ev)


def test_trace_roctx_ranges_load(monkeypatch):
    """With TV_ROCTX=1 spans become ROCTx ranges (no-ops without a profiler attached)."""
    from thinvids_amd.utils import trace

    if not os.path.exists("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"):
        pytest.skip("ROCm roctx library not installed")
    monkeypatch.setenv("TV_ROCTX", "1")
    monkeypatch.setattr(trace, "_roctx_tried", False)
    monkeypatch.setattr(trace, "_roctx", None)
    with trace.span("roctx.test"):
        pass
    assert trace._roctx is not None
