"""The 256x256 phased bf16 GEMM (csrc/gemm8p.hip) against a PyTorch fp32 reference of the
same op on the bf16-rounded inputs: all four operand layouts (forward Linear, dX = dY W,
dW = dY^T X, and A M-major / B K-major), bf16 and fp32 outputs, ragged M / N tails, K
tails of the MN-major (token-reduction) operands, split-K slabs, and the fused epilogue
(bias + GELU + kept pre-activation + residual; backward GELU'; beta accumulate).
Tolerances: 1e-2 relative with a bf16 output (one bf16 rounding of C), 3e-3 with fp32."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")


@pytest.fixture(scope="module", params=[5, 6], ids=["gemm8p", "gemm8q"])
def ops(request):
    """Every test runs on both 256x256 kernels: the phased one-tile-per-WG kernel (5) and the
    persistent register-epilogue kernel (6; epilogues it does not take fall back to 5)."""
    from capk import _lib, ops as _ops
    lib = _lib.load()
    lib.capk_gemm_force_config(request.param)
    _ops.FORCED_CFG = request.param
    yield _ops
    lib.capk_gemm_force_config(-1)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-30))


def _operand(rows, cols, kmajor, g, scale=1.0):
    """Logical [rows, K=cols] operand stored K-major ([rows][cols]) or MN-major ([cols][rows])."""
    x = (torch.randn(rows, cols, device="cuda", generator=g) * scale).bfloat16()
    return x, (x if kmajor else x.t().contiguous())


@cuda
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(1000, 520, 640), (768, 256, 1152), (256, 264, 64)])
@pytest.mark.parametrize("out", [torch.bfloat16, torch.float32])
def test_layouts_and_tails(ops, ak, bk, M, N, K, out):
    from capk import _lib
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a, A = _operand(M, K, ak, g)
    b, B = _operand(N, K, bk, g, 1.0 / math.sqrt(K))
    C = torch.empty(M, N, device="cuda", dtype=out)
    ops.gemm(A, ak, B, bk, M, N, K, C, lda=A.stride(0), ldb=B.stride(0), ldc=C.stride(0))
    # (gemm8q falls back to gemm8p for K <= 64 and for a split-K padding a K-major operand)
    assert _lib.load().capk_gemm_last_config() in (ops.FORCED_CFG, 5)
    ref = a.float() @ b.float().t()
    assert _rel(C, ref) < (1e-2 if out == torch.bfloat16 else 3e-3), (ak, bk, M, N, K)


@cuda
@pytest.mark.parametrize("K", [1000, 50432 // 4])
def test_weight_gradient_split_k_with_token_tail(ops, K):
    """dW[N, Kd] = dY^T X with the token reduction K not a multiple of 64 (zero-filled tail)
    and long enough for split-K slabs; fp32 output accumulated with beta = 1."""
    g = torch.Generator(device="cuda").manual_seed(K)
    N, Kd = 768, 512
    dy = torch.randn(K, N, device="cuda", generator=g).bfloat16()
    x = torch.randn(K, Kd, device="cuda", generator=g).bfloat16()
    dw = torch.randn(N, Kd, device="cuda", generator=g)
    dw0 = dw.clone()
    ops.linear_dw(dy, x, dw, accumulate=True)
    ref = dw0 + dy.float().t() @ x.float()
    assert _rel(dw, ref) < 3e-3


@cuda
def test_fused_epilogues(ops):
    from capk._lib import ACT_GELU_ERF
    g = torch.Generator(device="cuda").manual_seed(7)
    M, N, K = 1100, 768, 768
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    res = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y = ops.linear(x, w, bias, residual=res, act=ACT_GELU_ERF, preact=pre)
    ref_pre = x.float() @ w.float().t() + bias
    assert _rel(pre, ref_pre) < 1e-2
    assert _rel(y, F.gelu(ref_pre) + res.float()) < 1e-2
    # bias + GELU with kept pre-activation and no residual (the FFN1 shape)
    y2 = ops.linear(x, w, bias, act=ACT_GELU_ERF, preact=pre)
    assert _rel(y2, F.gelu(ref_pre)) < 1e-2
    # backward: dX * gelu'(aux)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    dxa = ops.linear_dx(dy, w, act_bwd=ACT_GELU_ERF, aux=pre)  # N == K here: aux has dX's shape
    a = pre.float().requires_grad_(True)
    F.gelu(a).backward(dy.float() @ w.float())
    assert _rel(dxa, a.grad) < 1e-2


@cuda
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("K", [128, 192, 1000])
def test_many_items_per_workgroup(ops, ak, bk, K):
    """289 tiles (> 256 workgroups): the persistent kernel runs several items per WG with the
    next item's first K-tiles loaded under the previous item's last ones and its epilogue
    stores in flight; K = 128 is the shortest item (2 K-tiles), 1000 a K tail (MN-major)."""
    if (ak or bk) and K % 64:
        pytest.skip("K-major operands need K % 64 == 0 on the 256x256 kernels")
    g = torch.Generator(device="cuda").manual_seed(K + 2 * ak + bk)
    M, N = 17 * 256 - 40, 17 * 256 - 8
    a, A = _operand(M, K, ak, g)
    b, B = _operand(N, K, bk, g, 1.0 / math.sqrt(K))
    bias = torch.randn(N, device="cuda", generator=g)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ops.gemm(A, ak, B, bk, M, N, K, C, lda=A.stride(0), ldb=B.stride(0), ldc=C.stride(0), bias=bias)
    ref = a.float() @ b.float().t() + bias
    assert _rel(C, ref) < 1e-2
    # the rows / columns of every tile landed where they belong (not only on average)
    err = (C.float() - ref).abs().amax(dim=1)
    assert float(err.max()) < 0.05 * float(ref.abs().max()), int(err.argmax())


@cuda
def test_epilogue_variants_exact_layout(ops):
    """The register-direct epilogue's lane -> (row, column) map, checked element by element
    with exact small-integer operands (asymmetric, so a transposed or permuted store shows):
    plain, bias + residual, beta * C, dropout (mask from capk_dropout_mask), GELU with the
    act' side output (CAPK_ACT_DERIV) and the backward multiply by aux."""
    from capk._lib import ACT_BWD, ACT_DERIV, ACT_GELU_ERF
    g = torch.Generator(device="cuda").manual_seed(11)
    M, N, K = 3 * 256 + 72, 2 * 256 + 128, 128
    a = torch.randint(-2, 3, (M, K), device="cuda", generator=g).bfloat16()
    w = torch.randint(-2, 3, (N, K), device="cuda", generator=g).bfloat16()
    ref = a.float() @ w.float().t()  # exact in fp32 and in bf16 (|x| <= 512)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ops.gemm(a, True, w, True, M, N, K, C, lda=K, ldb=K, ldc=N)
    assert torch.equal(C.float(), ref)
    bias = torch.randint(-3, 4, (N,), device="cuda", generator=g).float()
    res = torch.randint(-8, 9, (M, N), device="cuda", generator=g).bfloat16()
    ops.gemm(a, True, w, True, M, N, K, C, lda=K, ldb=K, ldc=N, bias=bias, residual=res, ldr=N)
    assert torch.equal(C.float(), ref + bias + res.float())
    C0 = torch.randint(-8, 9, (M, N), device="cuda", generator=g).bfloat16()
    C.copy_(C0)
    ops.gemm(a, True, w, True, M, N, K, C, lda=K, ldb=K, ldc=N, beta=1.0)
    assert torch.equal(C.float(), ref + C0.float())
    # dropout: keep mask of index m * N + n, scale 2 (p = 0.5)
    from capk import _lib
    mask = torch.empty(M * N, device="cuda", dtype=torch.uint8)
    L = _lib.load()
    _lib.check(L.capk_dropout_mask(M * N, 0, 0.5, 1234, mask.data_ptr(), ops._stream()), "capk_dropout_mask")
    ops.gemm(a, True, w, True, M, N, K, C, lda=K, ldb=K, ldc=N, drop=(0.5, 1234))
    assert torch.equal(C.float(), ref * 2.0 * mask.view(M, N).float())
    # forward GELU with act'(pre) kept; backward multiply by aux
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y = ops.linear(x, w, bias, act=ACT_GELU_ERF | ACT_DERIV, preact=pre)
    z = (x.float() @ w.float().t() + bias).requires_grad_(True)
    F.gelu(z).sum().backward()
    assert _rel(y, F.gelu(z.detach())) < 1e-2 and _rel(pre, z.grad) < 1e-2
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    wt = torch.randn(N, N, device="cuda", generator=g).bfloat16() / 16
    dx = ops.linear_dx(dy, wt, act_bwd=ACT_GELU_ERF | ACT_DERIV, aux=pre)
    assert _rel(dx, (dy.float() @ wt.float()) * pre.float()) < 1e-2


@cuda
@pytest.mark.parametrize("M", [6400 - 24, 1000])
def test_dx_act_colsum_fused(M):
    """capk_gemm_dx_act_colsum: C = (dY W) * act'(pre) with db = column sums of C, vs torch fp32
    on the bf16 inputs.  M = 6376 x N = 3072 is a persistent grid (25 x 12 items: the fused
    register-epilogue column sums, a ragged last tile row); M = 1000 takes the product +
    act_bwd_colsum route."""
    from capk import ops
    from capk._lib import ACT_DERIV, ACT_GELU_ERF
    g = torch.Generator(device="cuda").manual_seed(M)
    N, K = 3072, 768  # dX [M, N] = dY [M, K] @ W [K, N]
    dy = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(K, N, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    aux = torch.rand(M, N, device="cuda", generator=g).bfloat16()  # act'(pre) in [0, 1)
    db = torch.full((N,), 7.0, device="cuda")
    out = ops.linear_dx(dy, w, act_bwd=ACT_GELU_ERF | ACT_DERIV, aux=aux, dsum=db)
    ref = (dy.float() @ w.float()) * aux.float()
    assert _rel(out, ref) < 1e-2
    refb = out.float().sum(0)  # the sums of the values actually stored (bf16-rounded) ...
    assert _rel(db, ref.sum(0)) < 2e-3  # ... and of the exact product
    assert _rel(db, refb) < 2e-3


@cuda
@pytest.mark.parametrize("M", [6400 - 24, 1000])
def test_dx_act_colsum_weight_copy(M):
    """capk_gemm_dx_act_colsum_wt (W as its K-major copy, ops.WeightT): the same fused product
    and column sums as capk_gemm_dx_act_colsum on the N-major weight, both routes (persistent
    fused epilogue at M = 6376, product + act_bwd_colsum at M = 1000)."""
    from capk import ops
    from capk._lib import ACT_DERIV, ACT_GELU_ERF
    g = torch.Generator(device="cuda").manual_seed(M + 1)
    N, K = 3072, 768
    shadow = torch.zeros(K * N, device="cuda", dtype=torch.bfloat16)
    ops.WT.register(shadow)
    w = shadow.view(K, N)
    w.copy_((torch.randn(K, N, device="cuda", generator=g) / math.sqrt(K)).bfloat16())
    dy = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    aux = torch.rand(M, N, device="cuda", generator=g).bfloat16()
    res = {}
    ops.WT.MIN_ROWS = 1  # (instance override: the short product takes the copy too)
    for on in (True, False):
        ops.WT.enabled = on
        try:
            assert (ops.WT.get(w, M) is not None) == on
            db = torch.full((N,), 7.0, device="cuda")
            res[on] = (ops.linear_dx(dy, w, act_bwd=ACT_GELU_ERF | ACT_DERIV, aux=aux, dsum=db), db)
        finally:
            ops.WT.enabled = True
    del ops.WT.MIN_ROWS
    ref = (dy.float() @ w.float()) * aux.float()
    for on in (True, False):
        assert _rel(res[on][0], ref) < 1e-2
        assert _rel(res[on][1], ref.sum(0)) < 2e-3
    assert _rel(res[True][0], res[False][0]) < 1e-2


@cuda
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
def test_tail_round_exact(mode, ak, bk):
    """The persistent kernel's split-K tail round (capk_gemm_set_tail(1): after the whole
    round, the remaining row blocks run as K-splits into fp32 slabs, reduced with the epilogue by
    one more launch; 2: the split that arrives last at a tile sums the slabs and runs the
    epilogue inside the launch) vs whole items (0): a 273-item grid (21 x 13 tiles: 19 row blocks of whole
    items, 26 tail tiles x 3 splits) with K = 1536 (24 K-tiles, splits of 8), exact
    small-integer operands (every partial sum exact in fp32, so the slabs must reproduce the
    product bit for bit), plain / bias + residual / beta * C / GELU + act' / backward * aux
    epilogues, element by element; then two launches on one workspace."""
    from capk import _lib, ops
    from capk._lib import ACT_DERIV, ACT_GELU_ERF
    L = _lib.load()
    L.capk_gemm_force_config(6)
    L.capk_gemm_set_tail(mode)
    try:
        g = torch.Generator(device="cuda").manual_seed(21 + 2 * ak + bk)
        M, N, K = 20 * 256 + 72, 13 * 256, 1536
        a = torch.randint(-2, 3, (M, K), device="cuda", generator=g).bfloat16()
        w = torch.randint(-2, 3, (N, K), device="cuda", generator=g).bfloat16()
        A = a if ak else a.t().contiguous()
        B = w if bk else w.t().contiguous()
        ref = a.float() @ w.float().t()  # |x| <= 6144: exact in fp32; C = its bf16 rounding
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        kw = dict(lda=A.stride(0), ldb=B.stride(0), ldc=N)
        ops.gemm(A, ak, B, bk, M, N, K, C, **kw)
        assert L.capk_gemm_last_config() == 6
        assert torch.equal(C.float(), ref.bfloat16().float())
        bias = torch.randint(-3, 4, (N,), device="cuda", generator=g).float()
        res = torch.randint(-8, 9, (M, N), device="cuda", generator=g).bfloat16()
        ops.gemm(A, ak, B, bk, M, N, K, C, bias=bias, residual=res, ldr=N, **kw)
        assert torch.equal(C.float(), (ref + bias + res.float()).bfloat16().float())
        C0 = torch.randint(-8, 9, (M, N), device="cuda", generator=g).bfloat16()
        C.copy_(C0)
        ops.gemm(A, ak, B, bk, M, N, K, C, beta=1.0, **kw)
        assert torch.equal(C.float(), (ref + C0.float()).bfloat16().float())
        if ak and bk:  # forward activation (K-major only) and the backward multiply
            x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
            pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            y = ops.linear(x, w / 64, bias, act=ACT_GELU_ERF | ACT_DERIV, preact=pre)
            z = (x.float() @ (w.float() / 64).t() + bias).requires_grad_(True)
            F.gelu(z).sum().backward()
            assert _rel(y, F.gelu(z.detach())) < 1e-2 and _rel(pre, z.grad) < 1e-2
            aux = torch.randint(0, 3, (M, N), device="cuda", generator=g).bfloat16()
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            ops.gemm(a, True, w, True, M, N, K, out, lda=K, ldb=K, ldc=N, act=16 | ACT_GELU_ERF | ACT_DERIV, aux=aux,
                     ldx=N)
            assert torch.equal(out.float(), (ref * aux.float()).bfloat16().float())
        ws = torch.empty(L.capk_gemm_workspace(1, 1, M, N, K), dtype=torch.uint8, device="cuda")
        C1 = torch.empty_like(C)
        for _ in range(2):
            _lib.check(L.capk_gemm(1, 1, M, N, K, A.data_ptr(), A.stride(0), int(ak), B.data_ptr(), B.stride(0),
                                   int(bk), C1.data_ptr(), N, 1.0, 0.0, None, None, 0, 0, None, None, 0, 0.0, 0,
                                   ws.data_ptr(), ws.numel(), ops._stream()), "capk_gemm")
            assert torch.equal(C1.float(), ref.bfloat16().float())
    finally:
        L.capk_gemm_set_tail(-1)
        L.capk_gemm_force_config(-1)


@cuda
@pytest.mark.parametrize("out_f32", [False, True])
def test_tail_combine_matches_reduce(out_f32):
    """The in-launch tail combine (capk_gemm_set_tail(2): arrival tickets, the last split of a
    tail tile sums the slabs in split order and runs the register epilogue) against the reduce
    launch (1) on random operands: the same fp32 additions in the same order, so the outputs are
    bit-identical -- plain, bias + residual (bf16) / plain, bias (fp32 outputs), all four operand
    layouts, a 50 432 x 768 x 3072 ViT product (27 tail row blocks x 3 splits) and a 21 x 13-tile
    grid; repeated launches and a second stream (its own ticket block) included."""
    from capk import _lib, ops
    L = _lib.load()
    L.capk_gemm_force_config(6)
    try:
        g = torch.Generator(device="cuda").manual_seed(5)
        side = torch.cuda.Stream()
        for (M, N, K) in [(50432, 768, 3072), (20 * 256 + 72, 13 * 256, 1536)]:
            a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
            w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
            bias = torch.randn(N, device="cuda", generator=g)
            res = torch.randn(M, N, device="cuda", generator=g).bfloat16()
            layouts = [(True, True), (True, False), (False, True), (False, False)] if M < 50000 else [(True, True), (True, False)]
            for ak, bk in layouts:
                A = a if ak else a.t().contiguous()
                B = w if bk else w.t().contiguous()
                dt = torch.float32 if out_f32 else torch.bfloat16
                kw = dict(lda=A.stride(0), ldb=B.stride(0), ldc=N)
                epis = [dict(), dict(bias=bias)] if out_f32 else [dict(), dict(bias=bias, residual=res, ldr=N)]
                for epi in epis:
                    outs = {}
                    for mode in (1, 2, 2):
                        L.capk_gemm_set_tail(mode)
                        C = torch.full((M, N), float("nan"), device="cuda", dtype=dt)
                        ops.gemm(A, ak, B, bk, M, N, K, C, **kw, **epi)
                        assert L.capk_gemm_last_config() == 6
                        outs.setdefault(mode, []).append(C)
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        C = torch.full((M, N), float("nan"), device="cuda", dtype=dt)
                        ops.gemm(A, ak, B, bk, M, N, K, C, **kw, **epi)
                    torch.cuda.current_stream().wait_stream(side)
                    outs[2].append(C)
                    for C in outs[2]:
                        assert torch.equal(C, outs[1][0]), (M, ak, bk, sorted(epi))
        torch.cuda.synchronize()
    finally:
        L.capk_gemm_set_tail(-1)
        L.capk_gemm_force_config(-1)


@cuda
@pytest.mark.parametrize("tail", [0, 1, 2])
@pytest.mark.parametrize("group", [0, 2, 8, -1])
def test_grouped_raster_exact(group, tail):
    """The persistent kernel's grouped raster (capk_gemm_set_group: tiles of the whole-item rows
    walked in groups of `group` row blocks, column-major inside a group; 0 = row-major, -1 =
    the automatic choice) only reorders the items: a 21 x 13-tile grid (groups 8, 8, 5 -- or
    8, 8, 3 over the 19 whole-item rows when the split-K tail round is on) with K = 1536 and
    exact small-integer operands must give the exact product on every layout, with bias +
    residual, and the fused dX x act' + column sums (DSUM) must give identical outputs and
    column sums under every raster."""
    from capk import _lib, ops
    from capk._lib import ACT_DERIV, ACT_GELU_ERF
    L = _lib.load()
    L.capk_gemm_force_config(6)
    L.capk_gemm_set_tail(tail)
    L.capk_gemm_set_group(group)
    try:
        g = torch.Generator(device="cuda").manual_seed(7)
        M, N, K = 20 * 256 + 72, 13 * 256, 1536
        a = torch.randint(-2, 3, (M, K), device="cuda", generator=g).bfloat16()
        w = torch.randint(-2, 3, (N, K), device="cuda", generator=g).bfloat16()
        ref = a.float() @ w.float().t()
        for ak, bk in [(True, True), (True, False), (False, True), (False, False)]:
            A = a if ak else a.t().contiguous()
            B = w if bk else w.t().contiguous()
            C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            ops.gemm(A, ak, B, bk, M, N, K, C, lda=A.stride(0), ldb=B.stride(0), ldc=N)
            assert L.capk_gemm_last_config() == 6
            assert torch.equal(C.float(), ref.bfloat16().float()), (ak, bk)
        bias = torch.randint(-3, 4, (N,), device="cuda", generator=g).float()
        res = torch.randint(-8, 9, (M, N), device="cuda", generator=g).bfloat16()
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ops.gemm(a, True, w, True, M, N, K, C, lda=K, ldb=K, ldc=N, bias=bias, residual=res, ldr=N)
        assert torch.equal(C.float(), (ref + bias + res.float()).bfloat16().float())
        # fp32 outputs (the LM-head weight gradient's form: both operands MN-major), with the
        # split-K tail round reduced by the fp32 reduce
        C32 = torch.empty(M, N, device="cuda", dtype=torch.float32)
        at, wt_ = a.t().contiguous(), w.t().contiguous()
        ops.gemm(at, False, wt_, False, M, N, K, C32, lda=at.stride(0), ldb=wt_.stride(0), ldc=N)
        assert L.capk_gemm_last_config() == 6
        assert torch.equal(C32, ref)
        # DSUM: dX = dY W (W [K', N'] N-major) times aux, plus the column sums (fixed order)
        dy = torch.randint(-2, 3, (M, K), device="cuda", generator=g).bfloat16()
        wt = torch.randint(-2, 3, (K, N), device="cuda", generator=g).bfloat16()
        aux = torch.randint(0, 3, (M, N), device="cuda", generator=g).bfloat16()
        outs = []
        for gm in (0, group):
            L.capk_gemm_set_group(gm)
            db = torch.zeros(N, device="cuda")
            out = ops.linear_dx(dy, wt, act_bwd=ACT_GELU_ERF | ACT_DERIV, aux=aux, dsum=db)
            assert L.capk_gemm_last_config() == 6
            outs.append((out, db))
        exact = ((dy.float() @ wt.float()) * aux.float()).bfloat16()
        assert torch.equal(outs[1][0], exact)
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    finally:
        L.capk_gemm_set_group(-2)
        L.capk_gemm_set_tail(-1)
        L.capk_gemm_force_config(-1)
