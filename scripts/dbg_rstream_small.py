import sys, numpy as np, torch
sys.path[:0]=['/root/repo','/root/repo/tcp-stack_amd','/root/repo/tests']
import tcpck
from oracle.ref16 import Ref16C
o=Ref16C()
ctx=tcpck.Context(0, probe=True)
count, L, variant = 1, 16, 0
rng = np.random.default_rng(L * 7 + count + variant)
a = rng.integers(0, 256, count * L + 32, dtype=np.uint8)
a[:L] = 0xFF
buf = torch.from_numpy(np.ascontiguousarray(a)).cuda()
for trial in range(3):
    for init in ("empty", "full", "zeros"):
        out = {"empty": torch.empty, "full": lambda n, **k: torch.full((n,), -7, **k), "zeros": torch.zeros}[init](count, dtype=torch.int16, device="cuda")
        ctx.batch_fixed_ex(0, buf.data_ptr(), L, L, count, out, 5, variant)
        torch.cuda.synchronize()
        print(trial, init, out.cpu().numpy().view(np.uint16), o.batch(a, stride=L, length=L, count=count, threads=8), flush=True)
# also through the seg kernel and stream kernel for comparison
for k, p in ((1, 2), (3, 0), (4, 0), (2, 16)):
    out = torch.empty(count, dtype=torch.int16, device="cuda")
    try:
        ctx.batch_fixed_ex(0, buf.data_ptr(), L, L, count, out, k, p)
        torch.cuda.synchronize()
        print("kernel", k, p, out.cpu().numpy().view(np.uint16))
    except Exception as e:
        print("kernel", k, p, "err", e)
