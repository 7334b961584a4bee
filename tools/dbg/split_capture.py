import os, sys, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mercury_amd import gpu as G
from oracle import oracle as O
os.environ["MCHECKSUM_GPU_LIGHT"] = "0"
os.environ["MCHECKSUM_GPU_SPLIT"] = "1"
host = O.splitmix_bytes(8 << 20, 31337)
dev = torch.cat([torch.from_numpy(host).cuda(), torch.zeros(64, dtype=torch.uint8, device="cuda")])
want = O.batch_fixed("crc64", host, 512 << 10, 512 << 10, 16, nthreads=8)
G.prepare("crc64")
out = torch.zeros(16, dtype=torch.int64, device="cuda")
G.checksum_fixed("crc64", dev, 512 << 10, count=16, out=out)
torch.cuda.synchronize()
print("eager ok", np.array_equal(G.as_unsigned(out), want))
s = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
    G.checksum_fixed("crc64", dev, 512 << 10, count=16, out=out)
for r in range(4):
    out.fill_(12345)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    got = G.as_unsigned(out)
    print("replay", r, "ok", np.array_equal(got, want), [hex(int(x)) for x in got[:3]], [hex(int(x)) for x in want[:3]])
# unsplit reference value of piece terms
os.environ["MCHECKSUM_GPU_SPLIT"] = "0"
o2 = G.checksum_fixed("crc64", dev, 512 << 10, count=16)
torch.cuda.synchronize()
print("unsplit ok", np.array_equal(G.as_unsigned(o2), want))
