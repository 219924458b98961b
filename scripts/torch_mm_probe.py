#!/usr/bin/env python3
"""Library baseline for the frame-parallel GEMM shapes at c2 (torch fp32 ->
hipBLASLt / rocBLAS, TF32 off) and the HBM write rate of an L x 2048 fill:
what the hand-written gemm_x6s routes are compared with.
Median of 20 launches, HIP events, microseconds."""
import torch
torch.backends.cuda.matmul.allow_tf32 = False
L=65583
def t(f, n=20):
    f(); torch.cuda.synchronize(); ts=[]
    for _ in range(n):
        a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
        a.record(); f(); b.record(); torch.cuda.synchronize(); ts.append(a.elapsed_time(b)*1e3)
    ts.sort(); return ts[len(ts)//2]
x=torch.randn(L,144,device='cuda'); w=torch.randn(2048,144,device='cuda'); bias=torch.randn(2048,device='cuda')
C=torch.empty(L,2048,device='cuda')
print('fill L x 2048', t(lambda: C.fill_(1.0)))
print('copy L x 2048', t(lambda: C.copy_(C)))
print('torch addmm xproj', t(lambda: torch.addmm(bias, x, w.t(), out=C)))
h=torch.randn(L,256,device='cuda'); wo=torch.randn(256,256,device='cuda'); Co=torch.empty(L,256,device='cuda')
print('torch mm offset-head', t(lambda: torch.mm(h, wo.t(), out=Co)))
dg=torch.randn(L,1024,device='cuda'); D=torch.empty(1024,256,device='cuda'); D2=torch.empty(1024,144,device='cuda')
print('torch mm dW_hh', t(lambda: torch.mm(dg.t(), h, out=D)))
print('torch mm dW_ih', t(lambda: torch.mm(dg.t(), x, out=D2)))
