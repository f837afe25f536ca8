"""Which multi-stream pattern breaks HIP-graph capture?  mode: A fork/join only, B + events inside
capture, C = B + backward, D = events created before capture + backward."""
import sys
import torch

mode = sys.argv[1]
torch.manual_seed(0)
lin0 = torch.nn.Linear(256, 256).cuda()
lin1 = torch.nn.Linear(256, 256).cuda()
x = torch.randn(64, 256, device="cuda")
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
pre_events = [torch.cuda.Event() for _ in range(4)]


def fwd():
    cur = torch.cuda.current_stream()
    s0.wait_stream(cur)
    s1.wait_stream(cur)
    hand = []
    with torch.cuda.stream(s0):
        for i, sp in enumerate(x.split(16)):
            a = lin0(sp)
            if mode != "A":
                ev = pre_events[i] if mode == "D" else torch.cuda.Event()
                ev.record(s0)
                hand.append((a, ev))
            else:
                hand.append((a, None))
    if mode == "A":
        s1.wait_stream(s0)
    outs = []
    with torch.cuda.stream(s1):
        for a, ev in hand:
            if ev is not None:
                s1.wait_event(ev)
            outs.append(lin1(a))
    cur.wait_stream(s0)
    cur.wait_stream(s1)
    out = torch.cat(outs).sum()
    if mode in ("C", "D"):
        out.backward()
    return out


side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        fwd()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out = fwd()
g.replay()
torch.cuda.synchronize()
print("mode", mode, "ok", out.item())
