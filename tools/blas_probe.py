import torch, time
torch.backends.cuda.matmul.allow_bf16_reduced_precision_reduction = True
shapes = [("qkv_fwd", 50432, 2304, 768), ("fc1_fwd", 50432, 3072, 768), ("fc2_fwd", 50432, 768, 3072),
          ("o_fwd", 50432, 768, 768), ("lm_head_fwd", 5120, 50304, 768)]
dev = "cuda"
for name, M, N, K in shapes:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(N, device=dev, dtype=torch.bfloat16)
    for tag, fn in (("linear", lambda: torch.nn.functional.linear(a, w, b)), ("mm", lambda: a @ w.t()),
                    ("dW(dy^T x)", lambda: (torch.randn(0) if False else None))):
        if fn() is None: continue
        for _ in range(3): fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(10): fn()
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{name:12s} {tag:10s} {ms*1e3:8.1f} us {2*M*N*K/ms/1e9:8.1f} TF/s", flush=True)
    # dW = dy^T x : [N, K] = [M,N]^T [M,K]
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    fn = lambda: dy.t() @ a
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(10): fn()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{name:12s} {'dW':10s} {ms*1e3:8.1f} us {2*M*N*K/ms/1e9:8.1f} TF/s", flush=True)
    # dX = dy W : [M,K] = [M,N][N,K]
    fn = lambda: dy @ w
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10): fn()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{name:12s} {'dX':10s} {ms*1e3:8.1f} us {2*M*N*K/ms/1e9:8.1f} TF/s", flush=True)
