"""train.py's progressive-head losses on the HIP kernels (losses.py / csrc/hgk_loss.hip; SURVEY
§8(f) row 4) vs the reference's own loss classes (tests/golden/losses_trainpy.npz: fp64 values and
input gradients of the fp32-rounded inputs). fp32 kernels: 1e-5 relative on the loss, 1e-6 abs on
gradients. The top-k selection itself: exact against torch.topk's value set."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from progressive_process_for_human_pose_estimation_amd import losses as Lo

pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = [("ce_boot_0.5", "logits"), ("ce_boot_0.05", "logits"), ("ce_mask", "logits"),
         ("mse_mask", "x"), ("mse_boot_0.5", "x"), ("mse_boot_0.1", "x")]


@pytest.mark.parametrize("tag,which", CASES)
def test_losses_vs_reference(tag, which):
    g = dict(np.load(os.path.join(GOLDEN, "losses_trainpy.npz")))
    cls = torch.from_numpy(g["cls"]).to(DEV)
    mask = torch.from_numpy(g["mask"]).to(DEV)
    tgt = torch.from_numpy(g["tgt"]).to(DEV)
    a = torch.from_numpy(g[which]).to(DEV).requires_grad_()
    fn = {"ce_boot_0.5": lambda: Lo.Costomer_CrossEntropyLoss()(a, cls, 0.5),
          "ce_boot_0.05": lambda: Lo.Costomer_CrossEntropyLoss()(a, cls, 0.05),
          "ce_mask": lambda: Lo.Costomer_CrossEntropyLoss_with_mask()(a, cls, mask),
          "mse_mask": lambda: Lo.Costomer_MSELoss_with_mask()(a, tgt, mask),
          "mse_boot_0.5": lambda: Lo.Costomer_MSELoss()(a, tgt, 0.5),
          "mse_boot_0.1": lambda: Lo.Costomer_MSELoss()(a, tgt, 0.1)}[tag]
    loss = fn()
    (loss * 3.0).backward()  # the incoming gradient scales the input gradient (device scalar)
    ref = float(g[tag + "_loss"])
    assert abs(float(loss.detach()) - ref) <= 1e-5 * abs(ref) + 1e-6, (float(loss.detach()), ref)
    np.testing.assert_allclose(a.grad.cpu().numpy(), 3.0 * g[tag + "_grad"], rtol=0, atol=3e-6)


@pytest.mark.parametrize("L,k", [(4096, 2048), (4096, 409), (1000, 1), (1000, 1000), (9216, 4608)])
def test_topk_select_matches_torch(L, k):
    from progressive_process_for_human_pose_estimation_amd import hgk as H
    gen = torch.Generator(device=DEV).manual_seed(L + k)
    v = torch.randn(3, L, device=DEV, generator=gen)
    v[1] = v[1].abs()
    v[2, ::7] = 0.5  # many ties
    sel = torch.empty(3, L, device=DEV)
    sums = torch.empty(3, device=DEV)
    H.check(H.lib().hgk_topk_select(H.stream_handle(), v.data_ptr(), 3, L, k, sel.data_ptr(),
                                    sums.data_ptr()))
    top, _ = torch.topk(v, k, dim=1)
    assert torch.equal(sel.sum(1), torch.full((3,), float(k), device=DEV))
    picked = torch.sort(torch.where(sel > 0, v, torch.full_like(v, -1e30)), dim=1, descending=True)[0][:, :k]
    assert torch.equal(picked, top)
    torch.testing.assert_close(sums, top.double().sum(1).float(), rtol=1e-6, atol=1e-5)
    # ties at the threshold: the lowest indices are taken
    thr = top[:, -1:]
    for r in range(3):
        tied = torch.nonzero(v[r] == thr[r]).flatten()
        need = k - int((v[r] > thr[r]).sum())
        assert torch.equal(sel[r, tied[:need]], torch.ones(need, device=DEV))
        assert float(sel[r, tied[need:]].sum()) == 0.0
