"""The directory-level drop-in on the GPU: wal.OpenAtIndex(dir, i).ReadAll()
through ewal_open_at_index + ewal_wal_readall, replaying the reference's own
directory tests (wal/wal_test.go) on files the product's writer made."""
import json
import os

import pytest

from oracle import oracle as O
from etcd_amd import _lib as L
from etcd_amd import wal as W

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))


def _dir_bytes(d, names):
    return b"".join(open(os.path.join(d, n), "rb").read() for n in names)


def test_recover_after_cut(ctx, tmp_path):
    """TestRecoverAfterCut (wal/wal_test.go:265-324)."""
    g = GOLD["recover_after_cut"]
    p = str(tmp_path / "waltest")
    w = W.Create(p, b"metadata")
    w.SaveEntry(W.Entry())
    w.Cut()
    for i in range(1, 10):
        w.SaveEntry(W.Entry(Index=i))
        w.Cut()
    w.Close()
    os.remove(os.path.join(p, W.walName(*g["removed"])))
    for i in range(10):
        if i in g["file_not_found_for"]:
            with pytest.raises(L.EwalError) as ei:
                W.OpenAtIndex(p, i, ctx)
            assert ei.value.status == L.ERR_FILE_NOT_FOUND
            continue
        assert i in g["ok_for"]
        wal = W.OpenAtIndex(p, i, ctx)
        md, st, ents = wal.ReadAll()
        assert md == b"metadata"
        assert [e.Index for e in ents] == list(range(i, 10))
        # the same bytes through the oracle
        names = sorted(n for n in os.listdir(p) if n.endswith(".wal"))
        k = W.searchIndex(names, i)[0]
        o = O.readall(_dir_bytes(p, names[k:]), i)
        assert o["status"] == O.OK and [e["index"] for e in o["ents"]] == [e.Index for e in ents]
        wal.Close()


def test_recover(ctx, tmp_path):
    """TestRecover (wal/wal_test.go:152-196): metadata, ents, last state wins."""
    g = GOLD["recover"]
    p = str(tmp_path / "w")
    w = W.Create(p, g["metadata"].encode())
    ents = [W.Entry(0, x["term"], x["index"], bytes.fromhex(x["data_hex"]) if x["data_hex"] else None)
            for x in g["ents"]]
    for e in ents:
        w.SaveEntry(e)
    for s in g["states"]:
        w.SaveState(W.HardState(s["term"], s["vote"], s["commit"]))
    w.Close()
    md, st, got = W.OpenAtIndex(p, 0, ctx).ReadAll()
    assert md == g["metadata"].encode()
    assert (st.Term, st.Vote, st.Commit) == tuple(g["want_state"][k] for k in ("term", "vote", "commit"))
    assert [(e.Index, e.Term, e.Data) for e in got] == [(e.Index, e.Term, e.Data) for e in ents]


def test_open_at_uncommitted_index(ctx, tmp_path):
    """TestOpenAtUncommittedIndex (wal/wal_test.go:326-351)."""
    p = str(tmp_path / "w")
    w = W.Create(p, None)
    w.SaveEntry(W.Entry(Index=0))
    w.Close()
    wal = W.OpenAtIndex(p, 1, ctx)
    with pytest.raises(L.EwalError) as ei:
        wal.ReadAll()
    assert ei.value.status == L.ERR_INDEX_NOT_FOUND


def test_open_at_index_and_cut(ctx, tmp_path):
    """TestOpenAtIndex (wal/wal_test.go:60-112) + TestCut (:114-150), then the
    cut WAL replayed from every index through the GPU."""
    p = str(tmp_path / "w")
    w = W.Create(p, b"md")
    w.SaveEntry(W.Entry())
    w.Cut()
    assert os.path.exists(os.path.join(p, GOLD["cut_names"]["after_first_cut"]))
    w.SaveEntry(W.Entry(0, 1, 1, b"\x01"))
    w.Cut()
    assert os.path.exists(os.path.join(p, GOLD["cut_names"]["after_second_cut"]))
    for i in range(2, 40):
        w.SaveEntry(W.Entry(0, 1, i, bytes([i]) * i))
        if i % 7 == 0:
            w.Cut()
    w.SaveState(W.HardState(1, 1, 39))
    w.Close()
    names = sorted(os.listdir(p))
    for i in range(0, 40):
        wal = W.OpenAtIndex(p, i, ctx)
        k = W.searchIndex(names, i)[0]
        assert wal.seq == W.parseWalName(names[-1])[0]
        md, st, ents = wal.ReadAll()
        o = O.readall(_dir_bytes(p, names[k:]), i)
        assert o["status"] == O.OK
        assert [e.Index for e in ents] == [e["index"] for e in o["ents"]] == list(range(i, 40))
        assert (st.Term, st.Vote, st.Commit) == (1, 1, 39) and md == b"md"
        wal.Close()
    # a torn tail on the last file: io.ErrUnexpectedEOF from ReadAll
    last = os.path.join(p, names[-1])
    b = open(last, "rb").read()
    open(last, "wb").write(b[:-3])
    with pytest.raises(L.EwalError) as ei:
        W.OpenAtIndex(p, 30, ctx).ReadAll()
    assert ei.value.status == L.ERR_UNEXPECTED_EOF
