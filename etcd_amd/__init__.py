"""etcd_amd -- MI355X-native engine for etcd's WAL replay-and-verify path.

Product layout:
  csrc/        HIP kernels (gfx950) + host C++ behind the C ABI in include/ewal.h
  libewal.so   built in-tree by build.sh
  wal.py       mirror of the reference `wal` package (OpenAtIndex/ReadAll/Create/...)
  snap.py      mirror of `snap.Snapshotter` (Load / snapNames / batch verify)
  raftcommit.py batched `raft.maybeCommit` (SoA arrays or 192-B group records)
  crc.py       `pkg/crc` digest (chained CRC-32C) over host or device buffers
  raftmsg.py   batched `raftpb.Message` decode (the /raft ingress)
  shard.py     per-rank shard assignment, the RCCL summary all-reduce and the
               torch.distributed exchange of ONE WAL's split ranges (C join)
  _lib.py      ctypes bindings of include/ewal.h
"""
from . import _lib  # noqa: F401  (fails loudly if libewal.so is missing)
from .wal import Context, OpenAtIndex, Create, Encoder, readall_bytes, synth_wal  # noqa: F401

__all__ = ["Context", "OpenAtIndex", "Create", "Encoder", "readall_bytes", "synth_wal"]
