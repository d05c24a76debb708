"""Calibration probe: device info + plain-torch ResNet-50 step time (channels_last bf16).
Used only to calibrate our own engine against the library path; not part of the framework."""
import time, torch, json, sys
print("device", torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))
import torch.nn as nn
def bottleneck(cin, mid, cout, stride):
    class B(nn.Module):
        def __init__(s):
            super().__init__()
            s.c1=nn.Conv2d(cin,mid,1,bias=False); s.b1=nn.BatchNorm2d(mid)
            s.c2=nn.Conv2d(mid,mid,3,stride,1,bias=False); s.b2=nn.BatchNorm2d(mid)
            s.c3=nn.Conv2d(mid,cout,1,bias=False); s.b3=nn.BatchNorm2d(cout)
            s.sc=None
            if stride!=1 or cin!=cout:
                s.sc=nn.Sequential(nn.Conv2d(cin,cout,1,stride,bias=False),nn.BatchNorm2d(cout))
        def forward(s,x):
            r=x if s.sc is None else s.sc(x)
            y=torch.relu(s.b1(s.c1(x))); y=torch.relu(s.b2(s.c2(y))); y=s.b3(s.c3(y))
            return torch.relu(y+r)
    return B()
layers=[nn.Conv2d(3,64,7,2,3,bias=False),nn.BatchNorm2d(64),nn.ReLU(),nn.MaxPool2d(3,2,1)]
cin=64
for mid,n,st in [(64,3,1),(128,4,2),(256,6,2),(512,3,2)]:
    for i in range(n):
        layers.append(bottleneck(cin,mid,mid*4,st if i==0 else 1)); cin=mid*4
layers += [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(2048,1000)]
m=nn.Sequential(*layers).cuda().to(memory_format=torch.channels_last)
opt=torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
B=int(sys.argv[1]) if len(sys.argv)>1 else 256
x=torch.randn(B,3,224,224,device='cuda').to(memory_format=torch.channels_last)
y=torch.randint(0,1000,(B,),device='cuda')
def step():
    with torch.autocast('cuda',dtype=torch.bfloat16):
        loss=nn.functional.cross_entropy(m(x),y)
    opt.zero_grad(set_to_none=True); loss.backward(); opt.step()
for _ in range(5): step()
K=int(sys.argv[2]) if len(sys.argv)>2 else 20
torch.cuda.synchronize(); t=time.time()
for _ in range(K): step()
torch.cuda.synchronize(); dt=(time.time()-t)/K
print(json.dumps({"torch_eager_resnet50_bs":B,"ms":dt*1e3,"img_s":B/dt}))
