"""Layout / scale probe of capk_gemm_f8 (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
import torch  # noqa: E402

from capk import ops  # noqa: E402

M = N = 256
K = 128


def f8(x):
    return x.to(torch.float8_e4m3fn).view(torch.uint8).cuda()


def deq(q):
    return q.cpu().view(torch.float8_e4m3fn).float()


def run(qa, sa, qb, sb):
    C = torch.empty(M, N, device="cuda")
    ops.gemm_f8(qa, sa, qb, sb, C)
    return C.cpu()


g = torch.Generator().manual_seed(0)
one = torch.full((M,), 127, dtype=torch.uint8, device="cuda")
a = torch.randint(-3, 4, (M, K), generator=g).float()
b = torch.randint(-3, 4, (N, K), generator=g).float()
C = run(f8(a), one, f8(b), one)
ref = a @ b.t()
print("unit scales: max abs err", float((C - ref).abs().max()), "ref max", float(ref.abs().max()))
# one-hot A: A[m, k] = 1 at k = m % K  -> C[m, n] = B[n, m % K]
a1 = torch.zeros(M, K)
a1[torch.arange(M), torch.arange(M) % K] = 1
bi = (torch.arange(N)[:, None] * 0 + torch.arange(K)[None, :]).float()  # B[n,k] = k (exact up to 15.. no)
# e4m3 exact integers only up to 16 -> encode k as k % 16 and k // 16 separately
for name, bb in (("k%16", (torch.arange(K) % 16).float().expand(N, K)), ("k//16", (torch.arange(K) // 16).float().expand(N, K)),
                 ("n%16", (torch.arange(N) % 16).float()[:, None].expand(N, K)), ("n//16", (torch.arange(N) // 16 % 16).float()[:, None].expand(N, K))):
    C = run(f8(a1), one, f8(bb.contiguous()), one)
    print(name, "C[0:20, 0] =", C[0:20, 0].int().tolist(), " C[0, 0:20] =", C[0, 0:20].int().tolist())
    print(name, "C[16:36,0] =", C[16:36, 0].int().tolist())
# scales: A row m scaled by 2^(m%4), B unit
sa = (127 + torch.arange(M) % 4).to(torch.uint8).cuda()
C = run(f8(a), sa, f8(b), one)
ref = (a * torch.pow(2.0, (torch.arange(M) % 4).float())[:, None]) @ b.t()
print("A row scales: max abs err", float((C - ref).abs().max()))
sb = (127 + torch.arange(N) % 4).to(torch.uint8).cuda()
C = run(f8(a), one, f8(b), sb)
ref = a @ (b * torch.pow(2.0, (torch.arange(N) % 4).float())[:, None]).t()
print("B row scales: max abs err", float((C - ref).abs().max()))
ratio = C / (a @ b.t())
print("B scale ratio row0 cols 0..16:", [round(float(x), 3) for x in ratio[0, :16]])
C = run(f8(a), sa, f8(b), one)
ratio = C / (a @ b.t())
print("A scale ratio col0 rows 0..16:", [round(float(x), 3) for x in ratio[:16, 0]])
print("A scale ratio rows 16..48 step 4:", [round(float(x), 3) for x in ratio[16:48:4, 0]])
