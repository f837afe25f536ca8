"""HIP-graph captured training steps (`utils/graphs.py`): a replayed step must be the same optimizer
step as the eager one (device-side Adam step counter, fresh inputs copied into the static buffers)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _step_fn(model, opt):
    from pytorchdistributed_amd.ops import cross_entropy

    def step(x, y):
        opt.zero_grad(set_to_none=True)
        loss = cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        return loss

    return step


@pytest.mark.parametrize("opt_name", ["Adam", "AdamW", "SGD"])
def test_graphed_resnet_step_matches_eager(opt_name):
    from pytorchdistributed_amd import optim
    from pytorchdistributed_amd.models.resnet import resnet50
    from pytorchdistributed_amd.utils.graphs import GraphedStep

    torch.manual_seed(0)
    base = resnet50(num_classes=10, dtype=torch.bfloat16).to("cuda")
    eager, graphed = base, copy.deepcopy(base)
    kw = dict(lr=1e-3) if opt_name != "SGD" else dict(lr=1e-2, momentum=0.9)
    oe = getattr(optim, opt_name)(eager.parameters(), **kw)
    og = getattr(optim, opt_name)(graphed.parameters(), **kw)
    g = torch.Generator(device="cuda").manual_seed(1)
    batches = [(torch.randn(8, 64, 64, 3, device="cuda", generator=g).to(torch.bfloat16),
                torch.randint(0, 10, (8,), device="cuda", generator=g)) for _ in range(6)]
    se, sg = _step_fn(eager, oe), _step_fn(graphed, og)
    # GraphedStep warms up twice on the first batch before capturing: mirror that in eager
    for _ in range(2):
        se(*batches[0])
    gstep = GraphedStep(sg, batches[0], warmup=2, optimizer=og)
    losses_e, losses_g = [], []
    for x, y in batches[1:]:
        losses_e.append(se(x, y).float().item())
        losses_g.append(gstep(x, y).float().item())
    torch.cuda.synchronize()
    for a, b in zip(losses_e, losses_g):
        assert abs(a - b) <= 1e-3 * max(1.0, abs(a)), (losses_e, losses_g)
    for (n, pe), pg in zip(eager.named_parameters(), graphed.parameters()):
        err = ((pe.float() - pg.float()).norm() / (pe.float().norm() + 1e-12)).item()
        assert err < 1e-2, (n, err)
    # host-side step counters follow the replays (checkpoints record the true step)
    steps_e = sorted({s["step"] for s in oe.state.values() if "step" in s})
    steps_g = sorted({s["step"] for s in og.state.values() if "step" in s})
    assert steps_e == steps_g == [7]


def test_adam_device_step_counter_matches_host():
    """The device-counter path of adam_step must match the host-step path (bias corrections are
    evaluated with device powf instead of host powf: equal up to float rounding)."""
    from pytorchdistributed_amd._native import C

    torch.manual_seed(0)
    n = 4096
    w0 = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda")
    outs = []
    for use_dev in (False, True):
        w, m, v = w0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
        for t in range(1, 6):
            st = torch.full((1,), float(t), device="cuda") if use_dev else None
            C().adam_step(w, None, g, m, v, 1e-2, 0.9, 0.999, 1e-8, 0.0, False, t if not use_dev else 0, 1.0,
                          None, None, st)
        outs.append(w)
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-5, atol=1e-6)
