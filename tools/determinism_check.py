import copy, torch, sys
sys.path.insert(0, "/root/repo")
from pytorchdistributed_amd import optim
from pytorchdistributed_amd.models.resnet import resnet50
from pytorchdistributed_amd.ops import cross_entropy
torch.manual_seed(0)
base = resnet50(num_classes=10, dtype=torch.bfloat16).to("cuda")
a, b = base, copy.deepcopy(base)
oa, ob = optim.Adam(a.parameters(), lr=1e-3), optim.Adam(b.parameters(), lr=1e-3)
g = torch.Generator(device="cuda").manual_seed(1)
batches = [(torch.randn(8, 64, 64, 3, device="cuda", generator=g).to(torch.bfloat16),
            torch.randint(0, 10, (8,), device="cuda", generator=g)) for _ in range(4)]
for x, y in batches:
    for m, o in ((a, oa), (b, ob)):
        o.zero_grad(set_to_none=True)
        l = cross_entropy(m(x), y); l.backward(); o.step()
torch.cuda.synchronize()
bad = [(n, (pa.float()-pb.float()).abs().max().item()) for (n, pa), pb in zip(a.named_parameters(), b.parameters()) if not torch.equal(pa, pb)]
print("eager-vs-eager differing params:", len(bad), bad[:5])
