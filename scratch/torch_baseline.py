# Quick PyTorch-only ResNet-50 baseline (NOT part of the framework): measures what stock
# torch ops (MIOpen conv, native BN) give on one MI355X so kernel work can be prioritised.
import time, torch, torch.nn as nn, torch.nn.functional as F, sys
class Bottleneck(nn.Module):
    def __init__(s, cin, mid, stride, down):
        super().__init__()
        s.c1=nn.Conv2d(cin,mid,1,bias=False); s.b1=nn.BatchNorm2d(mid)
        s.c2=nn.Conv2d(mid,mid,3,stride,1,bias=False); s.b2=nn.BatchNorm2d(mid)
        s.c3=nn.Conv2d(mid,mid*4,1,bias=False); s.b3=nn.BatchNorm2d(mid*4)
        s.down = nn.Sequential(nn.Conv2d(cin,mid*4,1,stride,bias=False), nn.BatchNorm2d(mid*4)) if down else None
    def forward(s,x):
        i = x if s.down is None else s.down(x)
        y=F.relu(s.b1(s.c1(x))); y=F.relu(s.b2(s.c2(y))); y=s.b3(s.c3(y))
        return F.relu(y+i)
class R50(nn.Module):
    def __init__(s):
        super().__init__()
        s.stem=nn.Sequential(nn.Conv2d(3,64,7,2,3,bias=False),nn.BatchNorm2d(64),nn.ReLU(),nn.MaxPool2d(3,2,1))
        L=[]; cin=64
        for mid,n,st in [(64,3,1),(128,4,2),(256,6,2),(512,3,2)]:
            for i in range(n):
                L.append(Bottleneck(cin,mid,st if i==0 else 1,i==0)); cin=mid*4
        s.layers=nn.Sequential(*L); s.fc=nn.Linear(2048,1000)
    def forward(s,x):
        x=s.layers(s.stem(x)); return s.fc(torch.flatten(F.adaptive_avg_pool2d(x,1),1))
mode=sys.argv[1]; bs=int(sys.argv[2]); steps=int(sys.argv[3]) if len(sys.argv)>3 else 20
torch.backends.cudnn.benchmark=True
m=R50().cuda()
if 'cl' in mode: m=m.to(memory_format=torch.channels_last)
if 'bf16pure' in mode: m=m.bfloat16()
opt=torch.optim.SGD(m.parameters(),lr=0.1,momentum=0.9,weight_decay=5e-5, foreach=True)
x=torch.randn(bs,3,224,224,device='cuda'); y=torch.randint(0,1000,(bs,),device='cuda')
if 'cl' in mode: x=x.to(memory_format=torch.channels_last)
if 'bf16pure' in mode: x=x.bfloat16()
def step():
    opt.zero_grad(set_to_none=True)
    if 'amp' in mode:
        with torch.autocast('cuda',dtype=torch.bfloat16): out=m(x)
    else: out=m(x)
    loss=F.cross_entropy(out.float(),y); loss.backward(); opt.step()
for _ in range(5): step()
torch.cuda.synchronize(); t=time.time()
for _ in range(steps): step()
torch.cuda.synchronize(); dt=(time.time()-t)/steps
print(f"{mode} bs={bs} ms/step={dt*1e3:.2f} img/s={bs/dt:.1f}", flush=True)
