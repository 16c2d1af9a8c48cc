"""Graph-captured drop-in calls (modules.py): the reference's own loop (try_with_torch.py:330-344:
model(x) -> 4x nn.MSELoss -> zero_grad -> backward -> torch.optim.Adam) on the HIP modules replays
a hipGraph of the forward and one of the backward from the second call on. Every result must be
bitwise that of the eager drop-in (graph_calls off): heatmaps, losses, parameters after Adam, BN
running statistics and num_batches_tracked, input gradients, eval-mode inference."""
import pytest
import torch
import torch.nn as nn

import progressive_process_for_human_pose_estimation_amd as P
from progressive_process_for_human_pose_estimation_amd import modules as M
from progressive_process_for_human_pose_estimation_amd.data import gaussian_targets, synthetic_images

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(graph, stacks=2, dtype=torch.bfloat16):
    torch.manual_seed(0)
    return P.creatModel(nStack=stacks).to(DEV).set_engine_dtype(dtype).set_graph_mode(graph)


def _loop(m, xs, t, steps):
    """the reference's training loop; per step: heatmaps, loss, flat parameters, BN buffers"""
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    crit = nn.MSELoss()
    rec = []
    for i in range(steps):
        outs = m(xs[i % len(xs)])
        loss = sum(crit(o, t) for o in outs)
        opt.zero_grad()
        loss.backward()
        opt.step()
        torch.cuda.synchronize()
        rec.append((torch.stack([o.detach() for o in outs]).cpu(), float(loss.detach()),
                    torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu(),
                    {k: v.detach().clone().cpu() for k, v in m.named_buffers()}))
    return rec


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_graph_dropin_bitwise_equals_eager(dtype):
    """4 steps (1 eager warm-up, capture + replay, 2 pure replays) on two different batches."""
    xs = [synthetic_images(4, 128, 128, seed=s).to(DEV) for s in (1, 2)]
    t = gaussian_targets(4, 17, 32)[0].to(DEV)
    mg, me = _model(True, dtype=dtype), _model(False, dtype=dtype)
    rg, re_ = _loop(mg, xs, t, 4), _loop(me, xs, t, 4)
    cache = M._GRAPHS.get(mg)
    assert cache and all(e.fwd is not None and e.bwd is not None for e in cache.values())
    assert M._GRAPHS.get(me) is None
    for i, ((hg, lg, pg, bg), (he, le, pe, be)) in enumerate(zip(rg, re_)):
        assert torch.equal(hg, he), f"step {i}: heatmaps differ"
        assert lg == le, (i, lg, le)
        assert torch.equal(pg, pe), f"step {i}: parameters after Adam differ"
        assert bg.keys() == be.keys()
        for k in bg:
            assert torch.equal(bg[k], be[k]), f"step {i}: buffer {k} differs"
    assert int(dict(mg.named_buffers())["hourglass1.residual_block.bn1.num_batches_tracked"]) > 4


def test_graph_dropin_input_gradient_and_grad_none():
    """dx through a graphed call equals the eager one; parameters the dataflow never reaches
    (square blocks' conv4) keep grad None, as in the reference."""
    res = []
    for graph in (True, False):
        m = _model(graph, stacks=1)
        for _ in range(3):
            x = synthetic_images(2, 128, 128, seed=5).to(DEV).requires_grad_(True)
            out = m(x)
            (out[0].square().mean()).backward()
        torch.cuda.synchronize()
        res.append((x.grad.clone().cpu(), m.hourglass1.residual_block.conv4.weight.grad,
                    m.hourglass1.residual_block.conv2.weight.grad.clone().cpu()))
    assert torch.equal(res[0][0], res[1][0])
    assert res[0][1] is None and res[1][1] is None
    assert torch.equal(res[0][2], res[1][2])


def test_graph_eval_inference_no_grad():
    """eval-mode forward under no_grad (the reference's inference timing, hourglass_compare.py:
    1263-1273) is graphed too; each call sees its own input."""
    mg, me = _model(True).eval(), _model(False).eval()
    with torch.no_grad():
        for s in (3, 4, 5, 6):
            x = synthetic_images(2, 128, 128, seed=s).to(DEV)
            a, b = mg(x), me(x)
            for u, v in zip(a, b):
                assert torch.equal(u, v)
    assert all(e.fwd is not None and e.bwd is None for e in M._GRAPHS[mg].values())


def test_graph_busy_entry_falls_back_to_eager():
    """two forwards of one signature before their backward (gradient accumulation over two
    micro-batches): the second runs eagerly while the first keeps the graph's activations."""
    xs = [synthetic_images(2, 128, 128, seed=s).to(DEV) for s in (7, 8)]
    t = gaussian_targets(2, 17, 32)[0].to(DEV)
    grads = []
    for graph in (True, False):
        m = _model(graph, stacks=1)
        for _ in range(3):
            m.zero_grad()
            l0 = nn.functional.mse_loss(m(xs[0])[0], t)
            l1 = nn.functional.mse_loss(m(xs[1])[0], t)
            (l0 + l1).backward()
        torch.cuda.synchronize()
        grads.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()
                                if p.grad is not None]).cpu())
    assert torch.equal(grads[0], grads[1])


def test_graph_signature_change_recaptures():
    """a new batch size is a new signature (its own warm-up and graphs); the old one is kept."""
    m = _model(True, stacks=1)
    for n in (2, 2, 4, 4, 2):
        out = m(synthetic_images(n, 128, 128, seed=n).to(DEV))
        out[0].sum().backward()
    torch.cuda.synchronize()
    ents = list(M._GRAPHS[m].values())
    assert len(ents) == 2 and all(e.bwd is not None for e in ents)


def test_graph_cache_key_covers_routes_and_bn_scalars():
    """A captured call froze the routes and BN momentum / eps in force at capture: changing any of
    them is a new signature (eager first call, own capture), never a replay of the old launches."""
    from progressive_process_for_human_pose_estimation_amd import engine as E
    from progressive_process_for_human_pose_estimation_amd import hgk as H
    x = synthetic_images(2, 128, 128, seed=9).to(DEV)
    m = _model(True, stacks=1)
    with torch.no_grad():
        m(x)
        m(x)
        assert m.graph_cache_info() == {"signatures": 1, "captured": 1, "max_captured": 2}
        with E.routing(twin=False):
            a = m(x)
            assert m.graph_cache_info()["signatures"] == 2
        with H.route(img=0):
            m(x)
            assert m.graph_cache_info()["signatures"] == 3
        bn = m.hourglass1.residual_block.bn1
        mom = bn.momentum
        bn.momentum = mom + 0.1
        m(x)
        assert m.graph_cache_info()["signatures"] == 4
        bn.momentum = mom
        b = m(x)   # back to the first signature: its graph replays
        assert m.graph_cache_info()["signatures"] == 4
    e = _model(False, stacks=1)
    with torch.no_grad():
        ref = e(x)
        with E.routing(twin=False):
            ref_single = e(x)
    assert all(torch.equal(u, v) for u, v in zip(a, ref_single))
    assert all(torch.equal(u, v) for u, v in zip(b, ref))


def test_graph_cache_evicts_beyond_max_captured():
    """Each captured signature holds a memory pool: with max_graphs=1 a second capture evicts the
    first; the default keeps two (train + eval)."""
    m = _model(True, stacks=1)
    m.set_graph_mode(True, max_graphs=1)
    for n in (2, 2, 4, 4):
        out = m(synthetic_images(n, 128, 128, seed=n).to(DEV))
        out[0].sum().backward()
    torch.cuda.synchronize()
    info = m.graph_cache_info()
    assert info["captured"] == 1 and info["max_captured"] == 1
    m.set_graph_mode(True)          # the default cap again (cache cleared)
    assert m.graph_cache_info()["max_captured"] == 1   # the per-model setting persists
    with pytest.raises(ValueError):
        m.set_graph_mode(True, max_graphs=0)
