"""Diagnostic: one HIP-graph replayed training step vs the same eager step, bit for bit."""
import copy, sys
import torch
sys.path.insert(0, "/root/repo")
from pytorchdistributed_amd import optim
from pytorchdistributed_amd.models.resnet import resnet50
from pytorchdistributed_amd.ops import cross_entropy
from pytorchdistributed_amd.utils.graphs import GraphedStep

use_opt = len(sys.argv) > 1 and sys.argv[1] == "opt"
torch.manual_seed(0)
a = resnet50(num_classes=10, dtype=torch.bfloat16).to("cuda")
b = copy.deepcopy(a)
oa, ob = optim.Adam(a.parameters(), lr=1e-3), optim.Adam(b.parameters(), lr=1e-3)
g = torch.Generator(device="cuda").manual_seed(1)
batches = [(torch.randn(8, 64, 64, 3, device="cuda", generator=g).to(torch.bfloat16),
            torch.randint(0, 10, (8,), device="cuda", generator=g)) for _ in range(3)]

def mk(m, o):
    def step(x, y):
        o.zero_grad(set_to_none=True)
        l = cross_entropy(m(x), y); l.backward()
        if use_opt:
            o.step()
        return l
    return step

sa, sb = mk(a, oa), mk(b, ob)
for _ in range(2):
    sa(*batches[0])
gs = GraphedStep(sb, batches[0], warmup=2, optimizer=ob)
for i, (x, y) in enumerate(batches[1:]):
    la = sa(x, y); lb = gs(x, y)
    torch.cuda.synchronize()
    print("step", i, "loss eager", la.item(), "graph", lb.item(), "equal", torch.equal(la, lb))
    nd = 0
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        if not torch.equal(pa.grad, pb.grad):
            nd += 1
            if nd <= 6:
                print("  grad differs", n, (pa.grad.float() - pb.grad.float()).abs().max().item(), pa.grad.float().abs().max().item())
        if not torch.equal(pa, pb) and nd <= 6:
            print("  param differs", n)
    print("  params with differing grads:", nd)
