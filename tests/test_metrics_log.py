"""MetricsLog: the background writer (client agents) keeps record order, survives an unserialisable record and
drains on close."""
import json

from fedmi.utils.metrics import MetricsLog


def test_background_writer_order_and_drain(tmp_path):
    m = MetricsLog(tmp_path / "m.jsonl", background=True)
    for i in range(500):
        m.write(event="round", round=i)
    m.write(event="bad", obj=object())         # not JSON-serialisable: logged as an error record
    m.write(event="round", round=500)
    m.close()
    rows = [json.loads(x) for x in (tmp_path / "m.jsonl").read_text().splitlines()]
    rounds = [r["round"] for r in rows if r.get("event") == "round"]
    assert rounds == list(range(501))
    assert any(r.get("event") == "metrics_error" for r in rows)
    assert m.count == 502 and len(m.records) == 502


def test_background_writer_flush(tmp_path):
    m = MetricsLog(tmp_path / "m.jsonl", background=True)
    m.write(event="x", v=1)
    m.flush()
    assert json.loads((tmp_path / "m.jsonl").read_text().splitlines()[0])["v"] == 1
    m.close()
