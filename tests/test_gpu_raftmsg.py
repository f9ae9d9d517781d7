"""GPU parity of the batched raftpb.Message decode
against the oracle's restatement of Message.Unmarshal
(raft/raftpb/raft.pb.go:407-617).  The reference holds no Message test
vectors, so the random and hand-built bodies here are the pinning (the
oracle's marshal is MessageTo, raft.pb.go:1010-1068, round-tripped in
tests/test_oracle_golden.py)."""
import random

import pytest

from oracle import oracle as O
from etcd_amd import _lib as L
from etcd_amd import raftmsg as M

pytestmark = pytest.mark.gpu


def _rand_msg(rng):
    ents = [O.entry_marshal(rng.choice([0, 1]), rng.randrange(1 << rng.choice([3, 30, 63])), rng.randrange(1 << 40),
                            bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 50, 700]))))
            for _ in range(rng.choice([0, 0, 1, 3, 20]))]
    snap = O.snapshot_marshal(bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 10, 3000]))),
                              [rng.randrange(1, 1 << 20) for _ in range(rng.randrange(0, 4))],
                              rng.randrange(1 << 30), rng.randrange(1 << 10))
    return O.message_marshal(rng.randrange(16), rng.randrange(1 << 62), rng.randrange(1 << 62), rng.randrange(1 << 30),
                             rng.randrange(1 << 30), rng.randrange(1 << 40), ents, rng.randrange(1 << 40), snap,
                             rng.random() < 0.5)


def _check(ctx, bodies):
    got = M.decode_messages(ctx, bodies)
    for b, g in zip(bodies, got):
        o = O.message_unmarshal(bytes(b))
        assert g["status"] == o["status"], (g["status"], o["status"], bytes(b).hex())
        for k in ("type", "to", "from_", "term", "log_term", "index", "commit", "reject", "unrec", "unrec_len"):
            assert g[k] == o[k], k
        assert [(e["type"], e["term"], e["index"], e["data"], e["unrec"]) for e in g["ents"]] == \
            [(e["type"], e["term"], e["index"], e["data"], e["unrec"]) for e in o["ents"]]
        for k in ("data", "index", "term", "n_nodes", "n_removed", "unrec", "nodes", "removed"):
            assert g["snap"][k] == o["snap"][k], k
    return got


def test_messages_round_trip(ctx):
    rng = random.Random(41)
    bodies = [_rand_msg(rng) for _ in range(300)]
    got = _check(ctx, bodies)
    assert all(g["status"] == L.OK for g in got)


def test_messages_corrupted(ctx):
    rng = random.Random(42)
    bodies = []
    for i in range(400):
        b = bytearray(_rand_msg(rng))
        kind = i % 4
        if kind == 0 and b:
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        elif kind == 1:
            del b[rng.randrange(len(b) + 1):]
        elif kind == 2:
            b += bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 12)))
        else:
            p = rng.randrange(len(b))
            b[p:p] = bytes([rng.choice([0x3a, 0x4a, 0x58, 0x0b, 0x09, 0x0d]), 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                            0xff, 0xff, 0xff, 0x01])
        bodies.append(bytes(b))
    got = _check(ctx, bodies)
    assert len({g["status"] for g in got}) >= 3


def test_message_quirks(ctx):
    # an Entry whose Unmarshal fails is kept (error discarded, raft.pb.go:535)
    bad_entry = bytes([0x08, 0x01, 0x10])                 # truncated varint -> ErrUnexpectedEOF inside
    m1 = O.message_marshal(2, 1, 2, 3, 4, 5, [bad_entry, O.entry_marshal(0, 1, 9, b"ok")], 6, b"", False)
    # Reject is assigned, not OR-ed: true then false
    m2 = O.message_marshal(0, 0, 0, 0, 0, 0, [], 0, b"", True) + bytes([0x50, 0x00])
    # repeated Snapshot fields accumulate into one struct
    m3 = O.message_marshal(0, 0, 0, 0, 0, 0, [], 0, O.snapshot_marshal(b"", [1], 5, 0), False) + \
        bytes([0x4a, 0x02, 0x20, 0x07])
    # unknown message field -> XXX_unrecognized
    m4 = O.message_marshal(1, 1, 1, 1, 1, 1, [], 1, b"", False) + bytes([0x60, 0x05])
    # wrong wire type / empty body
    m5 = bytes([0x0a, 0x00])
    got = _check(ctx, [m1, m2, m3, m4, m5, b""])
    assert got[0]["status"] == L.OK and len(got[0]["ents"]) == 2
    assert got[1]["reject"] is False
    assert got[2]["snap"]["index"] == 5 and got[2]["snap"]["term"] == 7
    assert got[3]["status"] == L.OK and got[3]["unrec"] == bytes([0x60, 0x05])
    assert got[4]["status"] == L.ERR_WRONG_TYPE and got[5]["status"] == L.OK


def test_message_residual_encodings(ctx):
    """Values Go assembles by append: every XXX_unrecognized, Entry.Data and
    Snapshot.Data repeated with several non-empty segments, Nodes /
    RemovedNodes over repeated Snapshot fields and packed-free repeats."""
    unk = bytes([0x78, 0x2a]) + bytes([0x82, 0x01, 0x03]) + b"abc"       # fields 15 (varint), 16 (bytes)
    e_split = O.entry_marshal(0, 3, 7, b"head") + bytes([0x22, 0x04]) + b"tail" + unk
    e_empty_rep = O.entry_marshal(1, 3, 8, b"x") + bytes([0x22, 0x00])  # an empty repeat keeps the value
    snap = O.snapshot_marshal(b"part1", [4, 5], 9, 2) + bytes([0x0a, 0x05]) + b"part2" + unk
    snap2 = bytes([0x28, 0x0b, 0x10, 0x06, 0x0a, 0x00]) + unk           # RemovedNodes, another node, empty Data
    m = O.message_marshal(3, 1, 2, 4, 5, 6, [e_split, e_empty_rep], 7, snap, True) + \
        bytes([0x4a, len(snap2)]) + snap2 + unk + bytes([0x3a, len(e_split)]) + e_split
    many = O.snapshot_marshal(b"d", list(range(1, 200)), 1, 1)          # > 64 nodes
    m2 = O.message_marshal(1, 1, 1, 1, 1, 1, [], 1, many, False)
    got = _check(ctx, [m, m2])
    assert all(g["status"] == L.OK for g in got)
    g = got[0]
    assert g["ents"][0]["data"] == b"headtail" and g["ents"][0]["unrec"] == unk
    assert g["snap"]["data"] == b"part1part2" and g["snap"]["nodes"] == [4, 5, 6] and g["snap"]["removed"] == [11]
    assert g["unrec"] == unk and len(g["ents"]) == 3
    assert got[1]["snap"]["nodes"] == list(range(1, 200))


def test_message_residual_random(ctx):
    """Random bodies with unknown fields spliced in at field boundaries of
    the Message, its Entries and its Snapshot, and bytes fields repeated."""
    rng = random.Random(43)

    def unk():
        f = rng.choice([11, 12, 15, 100, 1000])
        wt = rng.choice([0, 1, 2, 5])
        tag = M._varint((f << 3) | wt)
        if wt == 0:
            return tag + M._varint(rng.randrange(1 << 40))
        if wt == 1:
            return tag + bytes(rng.getrandbits(8) for _ in range(8))
        if wt == 5:
            return tag + bytes(rng.getrandbits(8) for _ in range(4))
        d = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 20)))
        return tag + M._varint(len(d)) + d

    bodies = []
    for _ in range(300):
        ents = []
        for _ in range(rng.choice([0, 1, 3])):
            e = O.entry_marshal(0, rng.randrange(1 << 20), rng.randrange(1 << 20), b"a" * rng.randrange(0, 5))
            while rng.random() < 0.4:
                e += rng.choice([unk(), b"\x22" + M._varint(3) + b"xyz"])
            ents.append(e)
        sn = O.snapshot_marshal(b"s" * rng.randrange(0, 4), [rng.randrange(1, 99) for _ in range(rng.randrange(3))],
                                rng.randrange(99), rng.randrange(9))
        while rng.random() < 0.4:
            sn += rng.choice([unk(), b"\x0a\x02zz", b"\x10" + M._varint(rng.randrange(1, 1 << 30)),
                              b"\x28" + M._varint(rng.randrange(1, 1 << 30))])
        b = O.message_marshal(rng.randrange(16), 1, 2, 3, 4, 5, ents, 6, sn, False)
        while rng.random() < 0.5:
            b += unk()
        bodies.append(b)
    got = _check(ctx, bodies)
    assert all(g["status"] == L.OK for g in got)
