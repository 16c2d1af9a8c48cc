"""The progressive-head losses of the reference's train.py on HIP kernels (csrc/hgk_loss.hip;
SURVEY.md §8(f) row 4). Same names, constructor arguments and forward signatures as the reference:

    Costomer_CrossEntropyLoss()(input, target, fraction)        train.py:343-362
    Costomer_CrossEntropyLoss_with_mask()(input, target, mask)  train.py:365-376
    Costomer_MSELoss_with_mask()(input, target, mask)           train.py:379-391
    Costomer_MSELoss()(input, target, fraction)                 train.py:394-408

Inputs are the model's NCHW fp32 outputs on the GPU, class targets int64 [N, H, W], masks
[N, H, W] (any dtype; used as float). The bootstrapped losses keep the k = int(H * W * fraction)
largest per-pixel (or per-element) losses of each image, fraction clamped below at 0.1 (CE) /
0.25 (MSE) exactly as the reference; ties at the k-th value go to the lowest indices (torch.topk
leaves that order unspecified; the loss value does not depend on it). Everything, including the
backward, runs on libhgk kernels; only the final sum of N per-image sums is a torch op.
"""
import torch
import torch.nn as nn

from . import hgk as H


def _ptr(t):
    return None if t is None else t.data_ptr()


def _check_logits(x):
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4):
        raise H.HgkError("losses: expected a 4-D fp32 CUDA tensor [N, C, H, W]")
    return x.contiguous()


def _mask_f(mask, N, P):
    if mask is None:
        return None
    m = mask.reshape(N, P).to(torch.float32).contiguous()
    return m


class _PixelCE(torch.autograd.Function):
    """mean over the selected pixels of (mask *) CE; k = None: every pixel (divisor N*H*W)."""

    @staticmethod
    def forward(ctx, x, target, mask, k):
        x = _check_logits(x)
        N, K, Hh, W = x.shape
        P = Hh * W
        t = target.reshape(N, P).to(torch.int64).contiguous()
        mk = _mask_f(mask, N, P)
        lib, st = H.lib(), H.stream_handle()
        loss = torch.empty(N, P, device=x.device)
        bad = torch.zeros(1, dtype=torch.int32, device=x.device)
        H.check(lib.hgk_ce_pixels(st, x.data_ptr(), t.data_ptr(), _ptr(mk), N, K, P,
                                  loss.data_ptr(), bad.data_ptr()))
        kk = P if k is None else k
        sel = torch.empty(N, P, device=x.device)
        sums = torch.empty(N, device=x.device)
        H.check(lib.hgk_topk_select(st, loss.data_ptr(), N, P, kk, sel.data_ptr(), sums.data_ptr()))
        if int(bad.item()):
            raise H.HgkError("cross entropy: target class out of range")
        ctx.save_for_backward(x, t, sel, mk)
        ctx.denom = float(N * kk)
        ctx.k_all = k is None
        return sums.sum() / ctx.denom

    @staticmethod
    def backward(ctx, g):
        x, t, sel, mk = ctx.saved_tensors
        N, K, Hh, W = x.shape
        dx = torch.empty_like(x)
        gs = g.reshape(1).to(torch.float32).contiguous()
        H.check(H.lib().hgk_ce_grad(H.stream_handle(), x.data_ptr(), t.data_ptr(),
                                    None if ctx.k_all else sel.data_ptr(), _ptr(mk), N, K, Hh * W,
                                    gs.data_ptr(), 1.0 / ctx.denom, dx.data_ptr()))
        return dx, None, None, None


class _SqDiff(torch.autograd.Function):
    """mean over the selected elements of (mask *) (a - b)^2 per image; k = None: every element
    (divisor N*C*H*W)."""

    @staticmethod
    def forward(ctx, a, b, mask, k):
        a = _check_logits(a)
        b = b.to(torch.float32).contiguous()
        if b.shape != a.shape:
            raise H.HgkError("mse: target shape %s != input %s" % (tuple(b.shape), tuple(a.shape)))
        N, C, Hh, W = a.shape
        P = Hh * W
        mk = _mask_f(mask, N, P)
        lib, st = H.lib(), H.stream_handle()
        sq = torch.empty_like(a)
        H.check(lib.hgk_sqdiff(st, a.data_ptr(), b.data_ptr(), _ptr(mk), N, C, P, sq.data_ptr()))
        L = C * P
        kk = L if k is None else k
        sel = torch.empty(N, L, device=a.device)
        sums = torch.empty(N, device=a.device)
        H.check(lib.hgk_topk_select(st, sq.data_ptr(), N, L, kk, sel.data_ptr(), sums.data_ptr()))
        ctx.save_for_backward(a, b, sel, mk)
        ctx.denom = float(N * kk)
        ctx.k_all = k is None
        return sums.sum() / ctx.denom

    @staticmethod
    def backward(ctx, g):
        a, b, sel, mk = ctx.saved_tensors
        N, C, Hh, W = a.shape
        da = torch.empty_like(a)
        gs = g.reshape(1).to(torch.float32).contiguous()
        H.check(H.lib().hgk_sqdiff_grad(H.stream_handle(), a.data_ptr(), b.data_ptr(),
                                        None if ctx.k_all else sel.data_ptr(), _ptr(mk), N, C,
                                        Hh * W, gs.data_ptr(), 1.0 / ctx.denom, da.data_ptr()))
        return da, None, None, None


class Costomer_CrossEntropyLoss(nn.Module):  # noqa: N801 (reference name)
    """Bootstrapped pixel CE (train.py:343-362): mean of the k = int(H*W*max(fraction, 0.1))
    largest per-pixel CE losses of each image."""

    def __init__(self, weight=None, size_average=None, ignore_index=-100, reduce=None,
                 reduction="mean"):
        super().__init__()
        if weight is not None:
            raise NotImplementedError("class weights: the reference never sets them")
        self.ignore_index = ignore_index

    def forward(self, input, target, fraction):
        fraction = max(fraction, 0.1)
        k = int(input.shape[2] * input.shape[3] * fraction)
        return _PixelCE.apply(input, target, None, k)


class Costomer_CrossEntropyLoss_with_mask(nn.Module):  # noqa: N801
    """mean over N*H*W of CE * mask (train.py:365-376)."""

    def __init__(self, weight=None, size_average=None, ignore_index=-100, reduce=None,
                 reduction="mean"):
        super().__init__()
        self.ignore_index = ignore_index

    def forward(self, input, target, mask):
        return _PixelCE.apply(input, target, mask, None)


class Costomer_MSELoss_with_mask(nn.Module):  # noqa: N801
    """mean over N*C*H*W of (input - target)^2 * mask[:, None] (train.py:379-391)."""

    def __init__(self, weight=None, size_average=None, ignore_index=-100, reduce=None,
                 reduction="mean"):
        super().__init__()

    def forward(self, input, target, mask):
        return _SqDiff.apply(input, target, mask, None)


class Costomer_MSELoss(nn.Module):  # noqa: N801
    """Bootstrapped MSE (train.py:394-408): per image the k = int(H*W*max(fraction, 0.25))
    largest squared errors over its C*H*W elements, mean."""

    def __init__(self, weight=None, size_average=None, ignore_index=-100, reduce=None,
                 reduction="mean"):
        super().__init__()

    def forward(self, input, target, fraction):
        fraction = max(fraction, 0.25)
        k = int(input.shape[2] * input.shape[3] * fraction)
        return _SqDiff.apply(input, target, None, k)


def cross_entropy(input, target):
    """nn.CrossEntropyLoss()(input, target) for [N, K, H, W] logits (mean over pixels; -100
    ignored pixels count in the divisor here — the reference's targets never use it)."""
    return _PixelCE.apply(input, target, None, None)
