import copy, torch, sys
sys.path.insert(0, '/root/repo')
from pytorchdistributed_amd.models.resnet import resnet50
def rel(a, b): a, b = a.float().cpu(), b.float().cpu(); return ((a-b).norm()/(b.norm()+1e-12)).item()
torch.manual_seed(0)
cpu = resnet50(dtype=torch.bfloat16).float()
gpu = copy.deepcopy(cpu).to("cuda", torch.bfloat16)
x = torch.randn(4, 64, 64, 3).to(torch.bfloat16).float()
# stage by stage, feeding the CPU activation (rounded to bf16) into the GPU stage
a = x
for name, sc, sg in zip(["stem","layer1","layer2","layer3","layer4"], [cpu.stem, cpu.layer1, cpu.layer2, cpu.layer3, cpu.layer4],
                        [gpu.stem, gpu.layer1, gpu.layer2, gpu.layer3, gpu.layer4]):
    oc = sc(a)
    og = sg(a.to("cuda", torch.bfloat16))
    print(name, "rel", rel(og, oc), "norm", oc.norm().item())
    if name == "layer1":
        # block by block
        b = a if name != "stem" else None
    a = oc.to(torch.bfloat16).float()
# first bottleneck internals
blk_c, blk_g = cpu.layer1[0], gpu.layer1[0]
inp = cpu.stem(x).to(torch.bfloat16).float()
ig = inp.to("cuda", torch.bfloat16)
c1c = blk_c.conv1(inp); c1g = blk_g.conv1(ig); print("conv1", rel(c1g, c1c))
b1c = blk_c.bn1(c1c.to(torch.bfloat16).float(), relu=True); b1g = blk_g.bn1(c1c.to("cuda", torch.bfloat16), relu=True); print("bn1", rel(b1g, b1c))
dc = blk_c.downsample[0](inp); dg = blk_g.downsample[0](ig); print("ds conv", rel(dg, dc))
