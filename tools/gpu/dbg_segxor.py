# debug: decrypt of 4 KiB records through the records path, output pre-filled
# with 0xC3; classify every 1 KiB segment of every record
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "noise-cpp_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import noise_amd
noise_amd.load()
R, L = int(sys.argv[1]) if len(sys.argv) > 1 else 4096, int(sys.argv[2]) if len(sys.argv) > 2 else 4096
key = bytes(range(32))
d = np.zeros(R, dtype=noise_amd.record_dtype())
d["in_off"] = np.arange(R, dtype=np.uint64) * np.uint64(L)
d["out_off"] = np.arange(R, dtype=np.uint64) * np.uint64(L + 16)
d["nonce"] = np.arange(R, dtype=np.uint64)
d["len"] = L
dd = d.copy()
dd["in_off"], dd["out_off"] = d["out_off"], d["in_off"]
pt = torch.randint(0, 256, (R * L,), dtype=torch.uint8, device="cuda")
ct = torch.zeros(R * (L + 16), dtype=torch.uint8, device="cuda")
back = torch.full((R * L,), 0xC3, dtype=torch.uint8, device="cuda")
st = torch.full((R,), 9, dtype=torch.uint8, device="cuda")
k = torch.frombuffer(bytearray(key), dtype=torch.uint8).cuda()
noise_amd.encrypt_records(k, 1, torch.from_numpy(d.view(np.uint8).copy()).cuda(), R, pt, ct)
noise_amd.decrypt_records(k, 1, torch.from_numpy(dd.view(np.uint8).copy()).cuda(), R, ct, back, st)
torch.cuda.synchronize()
print("status values", torch.unique(st).tolist())
a = pt.cpu().numpy().reshape(R, L)
b = back.cpu().numpy().reshape(R, L)
nseg = L // 1024
cnt = {}
for s in range(nseg):
    seg_a, seg_b = a[:, 1024 * s:1024 * (s + 1)], b[:, 1024 * s:1024 * (s + 1)]
    ok = (seg_a == seg_b).all(axis=1)
    c3 = (seg_b == 0xC3).all(axis=1)
    z = (seg_b == 0).all(axis=1)
    print("segment %d: ok %d, untouched(C3) %d, zero %d, other %d" % (s, ok.sum(), c3.sum(), z.sum(), (~(ok | c3 | z)).sum()))
    bad = np.flatnonzero(~ok)[:8]
    print("   first bad records", bad.tolist())
w = back.cpu().numpy().view(np.uint32).reshape(-1, 4)
m = w[w[:, 0] & 0xFFFFFF00 == 0xFA11ED00]
if len(m):
    print("marks", len(m))
    for row in np.unique(m, axis=0)[:12]:
        print("  t %d fail_mask %08x%08x super0 %d" % (row[0] & 0xff, row[2], row[1], row[3]))
