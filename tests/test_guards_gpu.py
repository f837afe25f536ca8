"""Stream-safety guard: the fused optimizer refuses to update a flat gradient buffer
whose DDP bucket all-reduces the compute stream has not waited on yet."""
import pytest
import torch

from pytorchdistributed_amd.optim import SGD
from pytorchdistributed_amd.parallel.flat import FlatGroup

pytestmark = pytest.mark.gpu


def test_optimizer_refuses_unsynced_flat_grads():
    dev = torch.device("cuda", 0)
    params = [torch.nn.Parameter(torch.randn(64, 32, device=dev, dtype=torch.bfloat16)),
              torch.nn.Parameter(torch.randn(32, device=dev, dtype=torch.bfloat16))]
    fg = FlatGroup(params)
    fg.attach_grads()
    fg.grad_buffer.fill_(0.5)
    opt = SGD(params, lr=0.1, momentum=0.9)
    fg.pending_comm = 2  # as if two bucket collectives were still in flight
    with pytest.raises(RuntimeError, match="not waited on"):
        opt.step()
    fg.pending_comm = 0
    before = params[0].detach().float().clone()
    opt.step()
    torch.cuda.synchronize()
    assert not torch.equal(before, params[0].detach().float())
