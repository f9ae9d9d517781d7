import sys, os
sys.path.insert(0, os.getcwd())
order = sys.argv[1]
if order == "torch_first":
    import torch
    print("torch avail", torch.cuda.is_available(), torch.cuda.device_count())
    from etcd_amd import wal as W
else:
    from etcd_amd import wal as W
    import torch
    print("torch avail", torch.cuda.is_available(), torch.cuda.device_count())
buf, n = W.synth_wal(4 << 20, 64, 8192, seed=1)
r = W.readall_bytes(bytes(buf), 1)
print(order, "readall", r.status, r.n_records == n)
x = torch.ones(4, device="cuda"); torch.cuda.synchronize(); print("torch tensor ok", x.sum().item())
