import torch, time
dev='cuda'
def t(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e)/it
import os
M=int(os.environ.get("LP_B", "320"))*197
for k,n in [(768,2304),(768,768),(768,3072),(3072,768)]:
    x=torch.randn(M,k,device=dev,dtype=torch.bfloat16); w=torch.randn(n,k,device=dev,dtype=torch.bfloat16)
    ms=t(lambda: x@w.t()); print(f"torch bf16 {M}x{k}->{n}: {ms:.4f} ms {2*M*k*n/ms/1e9:.1f} TF/s", flush=True)
g=torch.randn(1600000,2048,device=dev,dtype=torch.bfloat16); q=torch.randn(320,2048,device=dev,dtype=torch.bfloat16)
ms=t(lambda: g@q.t(), 5); print(f"torch bf16 sweep 1.6Mx2048x320: {ms:.4f} ms {2*1.6e6*2048*320/ms/1e9:.1f} TF/s", flush=True)
x=torch.randn(8192,8192,device=dev,dtype=torch.bfloat16); y=torch.randn(8192,8192,device=dev,dtype=torch.bfloat16)
ms=t(lambda: x@y); print(f"torch bf16 8192^3: {ms:.4f} ms {2*8192**3/ms/1e9:.1f} TF/s", flush=True)
x=torch.randn(8192,8192,device=dev); y=torch.randn(8192,8192,device=dev)
ms=t(lambda: x@y,5); print(f"torch fp32 8192^3: {ms:.4f} ms {2*8192**3/ms/1e9:.1f} TF/s", flush=True)
