"""bench.py's exit code certifies every sub-line (CPU only: the workload
functions are replaced by stand-ins, no GPU call is made).  A sub-config that
raises -- its parity or gate asserts included (split2's join against the
oracle, rewind's n_ents, commit's record-vs-SoA check) -- still leaves the
headline line printed, names itself in `failed_configs`, and makes main()
return 1; a run whose sub-lines all finish returns 0 with every sub-line's
ms_per_step set."""
import json
import sys

import pytest

import bench


def _line(name):
    return {"metric": bench.METRIC, "value": 1.0, "unit": "GB/s", "ms_per_step": 1.5, "n_gpus": 1,
            "config": {"workload": name}}


@pytest.fixture
def fake_workloads(monkeypatch):
    monkeypatch.setattr(bench, "run_wal", lambda *a, **k: _line(k.get("label", "wal")))
    subs = {name: (lambda name: (lambda *a, **k: _line(name)))(name) for name in bench.SUBS if name != "c1"}
    subs["c1"] = None
    monkeypatch.setattr(bench, "SUBS", subs)
    return subs


def _main(monkeypatch, capsys, configs):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--configs", configs])
    rc = bench.main()
    out = capsys.readouterr().out.strip().splitlines()
    return rc, json.loads(out[-1])


def test_all_sub_lines_ok_exit_zero(fake_workloads, monkeypatch, capsys):
    rc, line = _main(monkeypatch, capsys, "c1,shards,snap,commit,rewind,split2")
    assert rc == 0
    assert "failed_configs" not in line
    assert set(line["configs"]) == {"c1", "shards", "snap", "commit", "rewind", "split2"}
    assert all(r["ms_per_step"] is not None for r in line["configs"].values())


def test_failed_sub_line_exits_nonzero(fake_workloads, monkeypatch, capsys):
    def broken(*a, **k):
        raise AssertionError("split2: join != oracle")   # a sub-line's parity gate

    fake_workloads["split2"] = broken
    rc, line = _main(monkeypatch, capsys, "c1,shards,split2,commit")
    assert rc == 1
    assert line["failed_configs"] == ["split2"]
    assert line["configs"]["split2"]["ms_per_step"] is None
    assert "AssertionError" in line["configs"]["split2"]["error"]
    # the other sub-lines and the headline are still reported
    assert line["ms_per_step"] == 1.5 and line["configs"]["commit"]["ms_per_step"] == 1.5
