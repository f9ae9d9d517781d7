"""k_fc ablation timing (diagnostic; results are wrong under ablation):
pipeline device ms of one ReadAll / one batched ReadAll per EWAL_FC_ABLATE
value (1 shift, 2 prefixes, 4 look-back, 8 ents stores, 16 no failure reports).
The product build ignores EWAL_FC_ABLATE: build the library with
-DEW_ABLATION_HOOKS (etcd_amd/build.sh -DEW_ABLATION_HOOKS) for these runs."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from etcd_amd import wal as W, _lib as L  # noqa: E402

variants = [int(x) for x in sys.argv[1].split(',')] if len(sys.argv) > 1 else [0, 16, 17, 18, 20, 24, 31]
blob, lens, _ = W.synth_shards(list(range(128)), 64 << 20, 128, 4096)
wal, _ = W.synth_wal(8 << 30, 64, 65536, seed=2)
for name, data in (("shards128", blob), ("wal8g", wal)):
    nb = len(data)
    c0 = W.Context(0)
    d = c0.alloc(nb + 64)
    d.upload_ptr(C.addressof((C.c_char * nb).from_buffer(data)), nb)
    for v in variants:
        os.environ["EWAL_FC_ABLATE"] = str(v)
        ctx = W.Context(0)
        ms = []
        for it in range(6):
            if name == "shards128":
                out = (L.Result * len(lens))()
                L.lib.ewal_readall_batch_device(ctx.handle, d.ptr, len(lens), (C.c_uint64 * len(lens))(*lens),
                                                (C.c_uint64 * len(lens))(*([1] * len(lens))), out)
                ms.append((out[0].device_ms, out[0].stream_ms))
            else:
                r = L.Result()
                L.lib.ewal_readall_device(ctx.handle, d.ptr, nb, 1, C.byref(r))
                ms.append((r.device_ms, r.stream_ms))
        ms = ms[2:]
        dev = sorted(x[0] for x in ms)[len(ms) // 2]
        st = sorted(x[1] for x in ms)[len(ms) // 2]
        print("%-10s ablate=%2d device_ms %.3f stream_ms %.3f post %.3f" % (name, v, dev, st, dev - st), flush=True)
        ctx.close()
    d.free()
    c0.close()
