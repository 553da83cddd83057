import torch
N,d=524288,768
x=torch.randn(N,d,device="cuda").bfloat16(); r=torch.randn(N,d,device="cuda").bfloat16(); o=torch.empty_like(x)
def t(fn,nb,name):
    for _ in range(3): fn()
    torch.cuda.synchronize(); e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): fn()
    e1.record(); torch.cuda.synchronize(); ms=e0.elapsed_time(e1)/20
    print(name, round(ms*1e3,1),"us", round(nb/(ms*1e-3)/1e12,2),"TB/s", flush=True)
t(lambda: o.copy_(x), 2*N*d*2, "copy")
t(lambda: torch.add(x,r,out=o), 3*N*d*2, "add")
