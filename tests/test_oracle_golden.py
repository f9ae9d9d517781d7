"""Pin the CPU oracle against the reference's own known-answer vectors.

tests/golden/reference_kats.json holds literals transcribed from the
reference's Go tests (citations inside).  The oracle is the checker for the
GPU engine, so it must reproduce every one of them first.
"""
import json
import os

import pytest

from oracle import oracle as O

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))


def test_crc32c_check_value():
    g = GOLD["crc32c_check"]
    d = bytes.fromhex(g["data_hex"])
    assert O.crc32_update(0, d) == g["crc"]
    assert O.crc32_update_table(0, d) == g["crc"]


def test_info_record_golden_bytes():
    g = GOLD["info_record"]
    info = bytes.fromhex(g["info_data_hex"])
    e = O.WalEncoder(0)
    e.encode(1, info)
    assert e.getvalue() == bytes.fromhex(g["record_hex"])
    # Crc field is crc32.Checksum(infoData, crcTable)
    assert O.record_unmarshal(bytes.fromhex(g["record_hex"])[8:])[1]["crc"] == O.crc32_update(0, info)


@pytest.mark.parametrize("case", GOLD["read_record_cases"]["cases"])
def test_read_record(case):
    rec = bytes.fromhex(GOLD["info_record"]["record_hex"])
    if case["cut"] == "all":
        data = rec
    elif case["cut"] == "bad":
        data = rec[:-1] + b"a"
    else:
        data = rec[:case["cut"]]
    st, r, _ = O.decode(data)[0]
    want = {"nil": O.OK, "io.EOF": O.EOF, "io.ErrUnexpectedEOF": O.ERR_UNEXPECTED_EOF,
            "walpb.ErrCRCMismatch": O.ERR_RECORD_CRC}[case["err"]]
    assert st == want
    if want == O.OK:
        assert r["type"] == case["type"] and r["data"] == bytes.fromhex(case["data_hex"])
    else:
        assert r == dict(type=0, crc=0, data=None)   # rec is the zero Record on error


def test_write_record_roundtrip():
    g = GOLD["write_record"]
    e = O.WalEncoder(0)
    e.encode(g["type"], g["data"].encode())
    st, r, _ = O.decode(e.getvalue())[0]
    assert st == O.OK and r["type"] == g["type"] and r["data"] == g["data"].encode()


def _recover_wal():
    g = GOLD["recover"]
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, g["metadata"].encode())
    for x in g["ents"]:
        e.save_entry(0, x["term"], x["index"], bytes.fromhex(x["data_hex"]) if x["data_hex"] else None)
    for s in g["states"]:
        e.save_state(s["term"], s["vote"], s["commit"])
    return e.getvalue()


def test_recover():
    g = GOLD["recover"]
    r = O.readall(_recover_wal(), 0)
    assert r["status"] == O.OK
    assert r["metadata"] == g["metadata"].encode()
    assert r["state"] == dict(g["want_state"], unrec=None)
    assert [(x["index"], x["term"], x["data"]) for x in r["ents"]] == \
        [(x["index"], x["term"], bytes.fromhex(x["data_hex"]) if x["data_hex"] else None) for x in g["ents"]]


def _cut_files():
    """TestRecoverAfterCut: files as (seq, index, bytes)."""
    files = []
    md = b"metadata"
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, md)
    e.save_entry(0, 0, 0, None)
    seq, enti = 0, 0
    name = (0, 0)
    for i in range(1, 10):
        files.append((name, e.getvalue()))
        prev = e.crc
        seq += 1
        name = (seq, enti + 1)
        e = O.WalEncoder(prev)
        e.save_crc(prev)
        e.encode(1, md)
        e.save_entry(0, 0, i, None)
        enti = i
    files.append((name, e.getvalue()))
    prev = e.crc
    name = (seq + 1, enti + 1)
    e = O.WalEncoder(prev)
    e.save_crc(prev)
    e.encode(1, md)
    files.append((name, e.getvalue()))
    return files


def test_recover_after_cut_chain():
    files = _cut_files()
    assert [f[0] for f in files[:3]] == [(0, 0), (1, 1), (2, 2)]
    whole = b"".join(f[1] for f in files)
    r = O.readall(whole, 0)
    assert r["status"] == O.OK and [x["index"] for x in r["ents"]] == list(range(10))
    for i in range(5, 10):
        tail = b"".join(f[1] for f in files if f[0][1] >= i or f[0] == (i, i))
        # the file whose start index <= i (searchIndex) and everything after it
        start = max(k for k, f in enumerate(files) if f[0][1] <= i)
        tail = b"".join(f[1] for f in files[start:])
        r = O.readall(tail, i)
        assert r["status"] == O.OK
        assert r["metadata"] == b"metadata"
        assert [x["index"] for x in r["ents"]] == list(range(i, 10))


def test_open_at_uncommitted_index():
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, None)
    e.save_entry(0, 0, 0, None)
    assert O.readall(e.getvalue(), 1)["status"] == O.ERR_INDEX_NOT_FOUND


@pytest.mark.parametrize("case", GOLD["commit"]["cases"])
def test_commit(case):
    rc, c = O.maybe_commit(case["matches"], case["smTerm"], 0, case["logs"])
    assert rc >= 0 and c == case["w"]


def test_log_at_bounds():
    g = GOLD["log_at"]
    terms = list(range(g["num"]))
    for tc in g["cases"]:
        i = tc["index"]
        # maybeCommit commits iff term(i) == term; term() is 0 when at() is nil
        want_term = 0 if tc["nil"] else i - g["offset"]
        rc, c = O.maybe_commit([i], want_term, 0, terms, g["offset"])
        assert c == (i if want_term == (0 if tc["nil"] else i - g["offset"]) and i > 0 else 0)
        if not tc["nil"]:
            rc2, c2 = O.maybe_commit([i], want_term + 1, 0, terms, g["offset"])
            assert c2 == 0


def test_snapshot_save_load_and_bad_crc():
    g = GOLD["snapshot"]["test_snap"]
    body = O.snapshot_marshal(g["data"].encode(), g["nodes"], g["index"], g["term"])
    f = O.snappb_marshal(O.crc32_update(0, body), body)
    r = O.loadsnap(f)
    assert r["status"] == O.OK
    assert r["snap"] == dict(data=g["data"].encode(), nodes=g["nodes"], index=g["index"], term=g["term"], removed=[],
                             unrec=None)
    # TestBadCRC: the table swapped to Koopman makes the stored CRC mismatch
    assert O.loadsnap(f, O.KOOPMAN)["status"] == O.ERR_SNAP_CRC
    # TestFailback: "bad data" is not a snappb.Snapshot
    assert O.loadsnap(GOLD["snapshot"]["failback_large_data"].encode())["status"] != O.OK


def test_decoder_eof_after_length_prefix():
    """io.ReadFull returns io.EOF (not ErrUnexpectedEOF) when zero payload
    bytes follow a length prefix (wal/decoder.go:35): ReadAll succeeds."""
    e = O.WalEncoder(0)
    e.save_crc(0)
    e.encode(1, b"m")
    w = e.getvalue() + (100).to_bytes(8, "little")
    assert O.readall(w, 0)["status"] == O.OK
    assert O.readall(w + b"x", 0)["status"] == O.ERR_UNEXPECTED_EOF


def test_skip_group_and_nontermination():
    # field 5 start-group ... end-group
    assert O.proto_skip(bytes([0x2B, 0x08, 0x01, 0x2C]))[0] == O.OK
    assert O.proto_skip(bytes([0x2B, 0x08, 0x01, 0x2C]))[1] == 4
    # unknown field 5 (wire 2) whose negative length makes skippy == 0: Go loops forever
    neg = lambda v: bytes([((2 ** 64 + v) >> (7 * k)) & 0x7F | (0x80 if k < 9 else 0) for k in range(10)])
    assert O.record_unmarshal(bytes([0x2A]) + neg(-11))[0] == O.NONTERMINATING
    # skippy < 0 -> data[index:index+skippy] slice-bounds panic
    assert O.record_unmarshal(bytes([0x2A]) + neg(-12))[0] == O.PANIC_BOUNDS
    # skippy > 0 but short: parsing resumes inside the length varint (0xFF 0x01 -> wire type 7)
    assert O.record_unmarshal(bytes([0x2A]) + neg(-2))[0] == O.ERR_WRONG_TYPE


def test_message_oracle_round_trip_and_quirks():
    """raftpb.Message restatement (raft/raftpb/raft.pb.go:407-617, 1010-1068)."""
    ents = [O.entry_marshal(0, 1, 5, b"hello"), O.entry_marshal(1, 2, 6, None)]
    snap = O.snapshot_marshal(b"xyz", [1, 2], 7, 3)
    m = O.message_marshal(3, 1, 2, 5, 4, 6, ents, 9, snap, True)
    # MarshalTo byte layout: fields 1-6, 7 per entry, 8, 9, 10 (raft.pb.go:1015-1063)
    assert m.hex() == ("0803100118022005280430063a0d080010011805220568656c6c6f3a08080110021806220040094a0d0a"
                       "0378797a10011002180720035001")
    d = O.message_unmarshal(m)
    assert d["status"] == O.OK and (d["type"], d["to"], d["from_"], d["term"], d["log_term"], d["index"],
                                    d["commit"], d["reject"]) == (3, 1, 2, 5, 4, 6, 9, True)
    assert [(e["term"], e["index"], e["data"]) for e in d["ents"]] == [(1, 5, b"hello"), (2, 6, None)]
    assert (d["snap"]["data"], d["snap"]["index"], d["snap"]["term"], d["snap"]["n_nodes"]) == (b"xyz", 7, 3, 2)
    # an Entry's Unmarshal error is discarded (:535): the message still decodes
    d = O.message_unmarshal(O.message_marshal(0, 0, 0, 0, 0, 0, [bytes([0x08, 0x01, 0x10])], 0, b"", False))
    assert d["status"] == O.OK and len(d["ents"]) == 1 and d["ents"][0]["type"] == 1
    # a panic inside it propagates (negative Data length -> slice bounds)
    neg = bytes([0x22]) + bytes([0xff] * 9) + bytes([0x01])
    assert O.message_unmarshal(bytes([0x3a, len(neg)]) + neg)["status"] == O.PANIC_BOUNDS
    # Reject is assigned; a negative embedded length panics; truncation -> ErrUnexpectedEOF
    assert O.message_unmarshal(bytes([0x50, 0x01, 0x50, 0x00]))["reject"] is False
    assert O.message_unmarshal(bytes([0x4a]) + bytes([0xff] * 9) + bytes([0x01]))["status"] == O.PANIC_BOUNDS
    assert O.message_unmarshal(m[:-1])["status"] == O.ERR_UNEXPECTED_EOF
    assert O.message_unmarshal(bytes([0x0a, 0x00]))["status"] == O.ERR_WRONG_TYPE
