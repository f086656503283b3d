"""Per-item timeline of the persistent GEMM (gemm8q) from the CAPK_DIAG_TRACE build
(scripts/build_diag.sh trace -> libcapk_diag_trace.so, loaded through CAPK_LIB_PATH).

Waves 0 (leading group) and 4 (lagging group) stamp s_memrealtime (100 MHz) at four points
of every item j: T2 first data wait of the item done, T3 first MFMA phase entered, T0 last
MFMA phase done, T1 epilogue done.  Per shape this prints medians over all WGs and items of
  main  = T0_j - T3_j  (the item's K loop)
  epi   = T1_j - T0_j  (epilogue: VALU + store issue; stores left in flight)
  wait  = T2_{j+1} - T1_j (next item's first operand wait, incl. stores counted ahead of it)
  sync  = T3_{j+1} - T2_{j+1} (barrier to the first MFMA phase)
and the launch span, for the leading group.

usage: CAPK_LIB_PATH=.../libcapk_diag_trace.so python tools/gemm_trace.py [name:M:N:K:kind,...]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from capk import _lib  # noqa: E402
import gemm_bench  # noqa: E402

DEFAULT = "qkv:50432:2304:768:fwd,fc1_plain:50432:3072:768:fwd,fc1g:50432:3072:768:fwd_gelu_deriv,o_res:50432:768:768:fwd_res,dx768:50432:768:768:dx,dx3072:50432:768:3072:dx,fc2dxg:50432:3072:768:dx_gelu_deriv"


def check_stamps(t, M, N, name):
    """Reject a trace with unwritten or stale slots (round 4's t17 run printed 9e16 us spans and
    the same item count for every shape): every WG must carry the item count its grid position
    gives (within one: the split-K tail round moves items), each stamped item all four stamps in the
    order T2 <= T3 <= T0 <= T1, consecutive items in order, and nothing past the item count."""
    items = ((M + 255) // 256) * ((N + 255) // 256)
    for w in range(256):
        first = (w & 7) * 32 + (w >> 3)
        expect = (items - first + 255) // 256 if first < items else 0
        for g in range(2):
            st = t[w, g]
            n = int((st[:, 0] > 0).sum())
            if not (max(0, expect - 1) <= n <= expect + 1) or (st[n:] != 0).any():
                raise SystemExit(f"{name}: WG {w} group {g}: {n} stamped items, expected {expect} -- stale trace")
            for j in range(n):
                a = st[j]
                if (a <= 0).any() or not (a[2] <= a[3] <= a[0] <= a[1]):
                    raise SystemExit(f"{name}: WG {w} group {g} item {j}: stamps {a.tolist()} unwritten / out of order")
                if j + 1 < n and st[j + 1, 2] < a[1]:
                    raise SystemExit(f"{name}: WG {w} group {g}: item {j + 1} starts before item {j} ends")


def main():
    spec = sys.argv[1] if len(sys.argv) > 1 else DEFAULT
    lib = _lib.load()
    fn = lib.capk_gemm_diag_trace  # (only in the diagnostic build)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros((256, 2, 64, 4), dtype=np.uint64)
    for item in spec.split(","):
        buf[:] = 0
        name, M, N, K, kind = item.split(":")
        gemm_bench.run(name, int(M), int(N), int(K), kind, iters=3)
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data, buf.nbytes) == 0
        t = buf.astype(np.int64)
        check_stamps(t, int(M), int(N), name)
        lead = t[:, 0]  # [WG, item, stamp]
        main_, epi, wait, sync = [], [], [], []
        for w in range(256):
            n = int((lead[w, :, 0] > 0).sum())
            for j in range(n):
                main_.append(lead[w, j, 0] - lead[w, j, 3])
                if j + 1 < n:
                    epi.append(lead[w, j, 1] - lead[w, j, 0])
                    wait.append(lead[w, j + 1, 2] - lead[w, j, 1])
                    sync.append(lead[w, j + 1, 3] - lead[w, j + 1, 2])
        valid = lead[lead > 0]
        span = (valid.max() - valid.min()) * 10 / 1000 if valid.size else 0
        med = lambda x: np.median(x) * 10 / 1000 if x else float("nan")  # us
        p90 = lambda x: np.percentile(x, 90) * 10 / 1000 if x else float("nan")
        print(f"{name:10s} items/WG {len(main_) / 256:4.1f}  main {med(main_):6.2f} us (p90 {p90(main_):6.2f})  "
              f"epi {med(epi):5.2f} (p90 {p90(epi):5.2f})  wait {med(wait):5.2f} (p90 {p90(wait):5.2f})  "
              f"sync {med(sync):5.2f}  span {span:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
