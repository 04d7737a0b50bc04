import torch
def bench(f, it=20):
    for _ in range(3): f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): f()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3
dev = "cuda"
# dW9^T[h][g] = sum_b A5^T[h][b] dL[b][g]  (M=1024, N=55039 (ld 55040), K=4096), fp32 out
A5 = (torch.rand(4096, 1024, device=dev) > 0.5).to(torch.bfloat16)
dL = (torch.randn(4096, 55040, device=dev) * 0.01).to(torch.bfloat16)
out = torch.empty(1024, 55040, device=dev, dtype=torch.float32)
try:
    us = bench(lambda: torch.mm(A5.t(), dL, out_dtype=torch.float32, out=out))
    print(f"dW9-like bf16->f32 out: {us:.1f} us {2*1024*55040*4096/us/1e6:.1f} TF/s")
except Exception as ex:
    print("out_dtype failed:", repr(ex)[:300])
    try:
        us = bench(lambda: torch.mm(A5.t(), dL, out_dtype=torch.float32))
        print(f"dW9-like bf16->f32 (alloc): {us:.1f} us")
    except Exception as ex2:
        print("out_dtype alloc failed:", repr(ex2)[:300])
us = bench(lambda: torch.mm(A5.t(), dL))
print(f"dW9-like bf16->bf16: {us:.1f} us")
X = (torch.rand(4096, 55040, device=dev) > 0.7).to(torch.bfloat16)
dY = (torch.randn(4096, 1024, device=dev) * 0.01).to(torch.bfloat16)
try:
    us = bench(lambda: torch.mm(dY.t(), X, out_dtype=torch.float32, out=out))
    print(f"dWe0-like bf16->f32 out: {us:.1f} us")
except Exception as ex:
    print("dWe0 out_dtype failed:", repr(ex)[:200])
