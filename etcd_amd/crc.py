"""pkg/crc mirror (pkg/crc/crc.go:15-41): a hash.Hash32 whose running value
starts at a previous CRC -- the chaining seed of the WAL decoder / encoder
(wal/decoder.go:24, wal/encoder.go:21).

`Write` takes host bytes (libewal's SSE4.2 / table path) or a DeviceBuffer
(one HBM stream pass on the GPU, ewal_crc32_update_device).  Every table Go's
crc32.MakeTable accepts works; the WAL uses Castagnoli (wal/wal.go:49).
"""
import ctypes as C
import struct

from . import _lib as L
from ._lib import lib, check


class Digest:
    """crc.New(prev, tab): Size 4, BlockSize 1, Reset -> 0 (not prev)."""

    def __init__(self, prev=0, poly=L.CASTAGNOLI):
        self.crc, self.poly = prev & 0xFFFFFFFF, poly

    def Write(self, data, n=None):
        """crc32.Update(d.crc, d.tab, p); data: bytes or a DeviceBuffer (n bytes)."""
        if hasattr(data, "ptr"):
            out = C.c_uint32()
            n = data.n if n is None else n
            check(lib.ewal_crc32_update_device(data.ctx.handle, self.crc, self.poly, data.ptr, n, C.byref(out)))
            self.crc = out.value
            return n
        b = bytes(data)
        self.crc = lib.ewal_crc32_update_host(self.crc, self.poly, b, len(b))
        return len(b)

    def Sum32(self):
        return self.crc

    def Sum(self, b=b""):
        """append(in, big-endian Sum32) (pkg/crc/crc.go:38-41)."""
        return bytes(b) + struct.pack(">I", self.crc)

    def Reset(self):
        self.crc = 0

    def Size(self):
        return 4

    def BlockSize(self):
        return 1


def New(prev, poly=L.CASTAGNOLI):
    return Digest(prev, poly)


def combine(crc_a, crc_b, len_b, poly=L.CASTAGNOLI):
    """Update(crc_a, B) from crc_b = Update(0, B) and len(B), bytes untouched."""
    return lib.ewal_crc32_combine(poly, crc_a, crc_b, len_b)
