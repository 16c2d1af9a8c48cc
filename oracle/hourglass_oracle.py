"""CPU ORACLE — test infrastructure only, never the product path.

A plain-PyTorch CPU restatement of the reference's stacked-hourglass hot path
(/root/reference/try_with_torch.py:179-298, and the nStack=1 / 18-output variant
/root/reference/only_one_hourgless.py:215-254). It is imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.

Parity pin: tests/golden/*.npz were generated from the reference's own classes (loaded by
tools/ref_loader.py, AST extraction, see tests/golden/make_golden.py); tests/test_oracle.py checks
this restatement against them (state_dict hash, outputs, grads, BN running stats).

Semantics reproduced exactly (SURVEY.md §0 "Semantics traps"):
  * one ResidualBlock object per hourglass level, reused for every up1/low1/low2/low3 call
    (try_with_torch.py:217,224-237); the same hourglass + residual4 + lin + heads for every stack
    (:268-273, :285-297) -> weight grads accumulate, BN running stats update once per use;
  * conv4 of a ResidualBlock is registered always (:193) but used only when numIn != numOut (:206);
  * pre-activation bottleneck BN->ReLU->1x1->BN->ReLU->3x3->BN->ReLU->1x1 (+skip) (:195-209);
  * bilinear x2 upsampling with align_corners=True, then up1 + up2 (:238-239);
  * MaxPool2d(2) down-sampling (:220,226,265);
  * heads conv2 (f->K), conv3 (f->f), conv4 (K->f), inter = conv3(ll) + conv4(out_k) (:291-297).
The parameter registration order equals the reference's, so torch.manual_seed(s) before
construction yields bit-identical initial weights (same kaiming-uniform draws in the same order).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class OracleResidual(nn.Module):
    # registration order: bn1, conv1, bn2, conv2, bn3, conv3, conv4  (try_with_torch.py:181-193)
    def __init__(self, cin, cout):
        super().__init__()
        mid = cout // 2
        self.numIn, self.numOut = cin, cout
        self.bn1 = nn.BatchNorm2d(cin)
        self.conv1 = nn.Conv2d(cin, mid, 1)
        self.bn2 = nn.BatchNorm2d(mid)
        self.conv2 = nn.Conv2d(mid, mid, 3, padding=1)
        self.bn3 = nn.BatchNorm2d(mid)
        self.conv3 = nn.Conv2d(mid, cout, 1)
        self.conv4 = nn.Conv2d(cin, cout, 1)

    def forward(self, x):
        h = self.conv1(F.relu(self.bn1(x)))
        h = self.conv2(F.relu(self.bn2(h)))
        h = self.conv3(F.relu(self.bn3(h)))
        skip = self.conv4(x) if self.numIn != self.numOut else x
        return h + skip


class OracleASPP(nn.Module):
    # try_with_aspp.py:195-207 — registered by the progressive preset's hourglass, never called
    # there; live at the innermost level of try_more_layer.py (:234-246): conv -> BN -> ReLU
    def __init__(self, inplanes, planes, k, padding, dilation):
        super().__init__()
        self.atrous_conv = nn.Conv2d(inplanes, planes, k, 1, padding, dilation, bias=False)
        self.bn = nn.BatchNorm2d(planes)

    def forward(self, x):
        return F.relu(self.bn(self.atrous_conv(x)))


class OracleHourglass(nn.Module):
    # try_with_torch.py:212-240 ; registration: residual_block, hourglass1 (if n>1), maxpool
    # (+ the dead ASPP branch of try_with_aspp.py:222-232 when aspp=True, same order)
    def __init__(self, n, f, n_modules=2, upsample="bilinear", aspp=False, aspp_live=False):
        super().__init__()
        self.n, self.f, self.n_modules, self.upsample = n, f, n_modules, upsample
        # try_more_layer.py:278-290: the innermost level runs the ASPP block (low2 = conv1(cat))
        self.aspp_live = aspp_live
        # try_with_aspp.py:245-246: no extra innermost residual chain in the ASPP variant
        self.inner_chain = not aspp
        self.residual_block = OracleResidual(f, f)
        if n > 1:
            self.hourglass1 = OracleHourglass(n - 1, f, n_modules, upsample, aspp, aspp_live)
        self.maxpool = nn.MaxPool2d(2)
        if aspp:
            self.aspp1 = OracleASPP(256, 256, 1, 0, 1)
            self.aspp2 = OracleASPP(256, 256, 3, 6, 6)
            self.aspp3 = OracleASPP(256, 256, 3, 12, 12)
            self.aspp4 = OracleASPP(256, 256, 3, 18, 18)
            self.global_avg_pool = nn.Sequential(nn.AdaptiveAvgPool2d((1, 1)),
                                                 nn.Conv2d(256, 256, 1, bias=False),
                                                 nn.BatchNorm2d(256), nn.ReLU())
            self.conv1 = nn.Conv2d(1280, 256, 1, bias=False)

    def _rb_chain(self, t):
        for _ in range(self.n_modules):
            t = self.residual_block(t)
        return t

    def forward(self, x):
        up1 = self._rb_chain(x)
        low = self._rb_chain(self.maxpool(x))
        if self.n > 1:
            low = self.hourglass1(low)
        elif self.aspp_live:
            parts = [m(low) for m in (self.aspp1, self.aspp2, self.aspp3, self.aspp4)]
            x5 = self.global_avg_pool(low)
            parts.append(F.interpolate(x5, size=low.shape[2:], mode="bilinear", align_corners=True))
            low = self.conv1(torch.cat(parts, dim=1))
        elif self.inner_chain:
            low = self._rb_chain(low)
        low = self._rb_chain(low)
        if self.upsample == "bilinear":
            up2 = F.interpolate(low, scale_factor=2, mode="bilinear", align_corners=True)
        else:
            up2 = F.interpolate(low, scale_factor=2, mode="nearest")
        return up1 + up2


class OracleLin(nn.Module):
    # try_with_torch.py:243-256 : 1x1 conv -> BN -> ReLU
    def __init__(self, cin, cout):
        super().__init__()
        self.numIn, self.numOut = cin, cout
        self.conv = nn.Conv2d(cin, cout, 1)
        self.bn = nn.BatchNorm2d(cout)

    def forward(self, x):
        return F.relu(self.bn(self.conv(x)))


class OracleModel(nn.Module):
    """creatModel restated (try_with_torch.py:259-298); nStack / nFeats / nOutChannels / nModules
    are the reference's module globals (:23-28), passed here as arguments."""

    def __init__(self, nStack=4, nFeats=256, nOutChannels=17, nModules=2, depth=4,
                 upsample="bilinear"):
        super().__init__()
        self.nStack, self.nModules = nStack, nModules
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3)
        self.residual1 = OracleResidual(64, 128)
        self.max_pool1 = nn.MaxPool2d(2)
        self.residual2 = OracleResidual(128, 128)
        self.residual3 = OracleResidual(128, nFeats)
        self.hourglass1 = OracleHourglass(depth, nFeats, nModules, upsample)
        self.residual4 = OracleResidual(nFeats, nFeats)
        self.lin = OracleLin(nFeats, nFeats)
        self.conv2 = nn.Conv2d(nFeats, nOutChannels, 1)
        self.conv3 = nn.Conv2d(nFeats, nFeats, 1)
        self.conv4 = nn.Conv2d(nOutChannels, nFeats, 1)

    def forward(self, x):
        x = F.relu(self.conv1(x))
        x = self.residual3(self.residual2(self.max_pool1(self.residual1(x))))
        heatmaps = []
        inter = x
        for s in range(self.nStack):
            ll = self.hourglass1(inter)
            for _ in range(self.nModules):
                ll = self.residual4(ll)
            ll = self.lin(ll)
            hm = self.conv2(ll)
            heatmaps.append(hm)
            # the reference also computes inter after the last stack (:294-297, `i < nStack` is
            # always true); it feeds nothing, so it cannot change any output or gradient.
            if s + 1 < self.nStack:
                inter = self.conv3(ll) + self.conv4(hm)
        return heatmaps


class OracleProgressive(nn.Module):
    """try_with_aspp.py:299-343 / try_different_stack.py:282-330 restated: primary trunk, 3 stacks, progressive heads
    conv2_0 (2, no bias) -> cat -> conv4_0 (258->256) ; conv2_1 (20, no bias) -> cat -> conv4_1
    (276->256, no bias) ; conv2_2 (17, no bias). Registration order as the reference's."""

    def __init__(self, nStack=3, nFeats=256, nModules=2, nOut=(2, 20, 17), depth=4, aspp=True,
                 aspp_live=False, late_heads=False):
        super().__init__()
        self.nStack, self.nModules = nStack, nModules
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3)
        self.residual1 = OracleResidual(64, 128)
        self.max_pool1 = nn.MaxPool2d(2)
        self.residual2 = OracleResidual(128, 128)
        self.residual3 = OracleResidual(128, nFeats)
        # aspp=True: try_with_aspp.py (dead ASPP registrations, no innermost chain);
        # aspp=False: try_different_stack.py:235-330 (primary hourglass)
        # aspp_live / late_heads: try_more_layer.py (live innermost ASPP; `elif i >= 2`, :355)
        self.hourglass1 = OracleHourglass(depth, nFeats, nModules, aspp=aspp, aspp_live=aspp_live)
        self.late_heads = late_heads
        self.residual4 = OracleResidual(nFeats, nFeats)
        self.lin = OracleLin(nFeats, nFeats)
        self.conv2_0 = nn.Conv2d(nFeats, nOut[0], 1, bias=False)
        self.conv4_0 = nn.Conv2d(nFeats + nOut[0], nFeats, 1)
        self.conv2_1 = nn.Conv2d(nFeats, nOut[1], 1, bias=False)
        self.conv4_1 = nn.Conv2d(nFeats + nOut[1], nFeats, 1, bias=False)
        self.conv2_2 = nn.Conv2d(nFeats, nOut[2], 1, bias=False)

    def forward(self, x):
        x = F.relu(self.conv1(x))
        inter = self.residual3(self.residual2(self.max_pool1(self.residual1(x))))
        heads = [(self.conv2_0, self.conv4_0), (self.conv2_1, self.conv4_1), (self.conv2_2, None)]
        out = []
        for i in range(self.nStack):
            ll = self.hourglass1(inter)
            for _ in range(self.nModules):
                ll = self.residual4(ll)
            ll = self.lin(ll)
            if i >= 3 and not self.late_heads:
                continue  # try_with_aspp.py `elif i == 2`: a 4th stack emits nothing
            head, back = heads[min(i, 2)]
            tmp = head(ll)
            out.append(tmp)
            if back is not None and i < 2:
                inter = back(torch.cat([ll, tmp], dim=1))
        return out


def progressive_loss(outs, bg, skeleton, keypoints):
    """try_with_aspp.py:393-396: CE(out0, bg) + CE(out1, skeleton) + MSE(out2, keypoints)."""
    return (F.cross_entropy(outs[0], bg) + F.cross_entropy(outs[1], skeleton)
            + F.mse_loss(outs[2], keypoints))


def stack_mse(heatmaps, target):
    """4x nn.MSELoss summed (try_with_torch.py:305-308,333-341): sum_s mean((o_s - t)^2)."""
    return sum(F.mse_loss(h, target) for h in heatmaps)


# ---------------------------------------------------------------------------------------------
# hourglass_compare.py preset: hourglass_compare.py:405-441 (block), :492-538
# (unshared hourglass, nearest up-sampling), :540-638 (stem with BN, 4 unshared stages, 16 heads)
class OracleCmpResidual(nn.Module):
    def __init__(self, numIn, numOut, stride=1):
        super().__init__()
        self.stride, self.numIn, self.numOut = stride, numIn, numOut
        mid = int(numOut / 2)
        self.bn1 = nn.BatchNorm2d(numIn)
        self.conv1 = nn.Conv2d(numIn, mid, 1, 1)
        self.bn2 = nn.BatchNorm2d(mid)
        self.conv2 = nn.Conv2d(mid, mid, 3, stride, 1)
        self.bn3 = nn.BatchNorm2d(mid)
        self.conv3 = nn.Conv2d(mid, numOut, 1, 1)
        self.bn4 = nn.BatchNorm2d(numOut)
        self.downsaple = nn.Sequential(nn.Conv2d(numIn, numOut, 1, stride=stride, bias=False),
                                       nn.BatchNorm2d(numOut))

    def forward(self, x):
        h = self.conv1(F.relu(self.bn1(x)))
        h = self.conv2(F.relu(self.bn2(h)))
        out = self.bn4(self.conv3(F.relu(self.bn3(h))))
        # hourglass_compare.py:438: `stride != 1 | numIn != numOut` parses as the chained
        # comparison stride != (1 | numIn) != numOut -> true for even channel counts
        residual = self.downsaple(x) if (self.stride != 1 | self.numIn != self.numOut) else x
        return out + residual


class OracleCmpHourglass(nn.Module):
    def __init__(self, f):
        super().__init__()
        for i in range(1, 5):
            setattr(self, f"downsample{i}", nn.Sequential(nn.MaxPool2d(2, 2), OracleCmpResidual(f, f)))
        for i in range(1, 6):
            setattr(self, f"residual{i}", OracleCmpResidual(f, f))
        for i in range(1, 5):
            setattr(self, f"upsample{i}", OracleCmpResidual(f, f))

    def forward(self, x):
        ups, d = [], x
        for i in range(1, 5):
            ups.append(getattr(self, f"residual{i}")(d))
            d = getattr(self, f"downsample{i}")(d)
        out = self.residual5(d)
        for i in (4, 3, 2, 1):
            out = getattr(self, f"upsample{i}")(out)
            out = F.interpolate(out, scale_factor=2) + ups[i - 1]
        return out


class OracleHGCompare(nn.Module):
    def __init__(self, nFeats=256, nOut=16):
        super().__init__()
        self.preprocess1 = nn.Sequential(
            nn.Conv2d(3, 64, 7, 2, 3), nn.BatchNorm2d(64), nn.ReLU(), OracleCmpResidual(64, 128),
            nn.MaxPool2d(2, 2), OracleCmpResidual(128, 128), OracleCmpResidual(128, nFeats))
        for k in range(1, 5):
            setattr(self, f"stage{k}", nn.Sequential(
                OracleCmpHourglass(nFeats), OracleCmpResidual(nFeats, nFeats),
                nn.Conv2d(nFeats, nFeats, 1, 1, 0), nn.BatchNorm2d(nFeats), nn.ReLU()))
            setattr(self, f"stage{k}_out", nn.Conv2d(nFeats, nOut, 1, 1, 0, bias=False))
            if k < 4:
                setattr(self, f"stage{k}_return", nn.Conv2d(nOut, nFeats, 1, 1, 0, bias=False))
                setattr(self, f"stage{k}_down_feature", nn.Conv2d(nFeats, nFeats, 1, 1, 0, bias=False))

    def forward(self, x):
        inter = self.preprocess1(x)
        out = []
        for k in range(1, 5):
            ll = getattr(self, f"stage{k}")(inter)
            tmp = getattr(self, f"stage{k}_out")(ll)
            out.append(tmp)
            if k < 4:
                inter = getattr(self, f"stage{k}_return")(tmp) + inter + \
                    getattr(self, f"stage{k}_down_feature")(ll)
        return out


# ---------------------------------------------------------------- train.py (stride-2 blocks)
class OracleTrainASPP(nn.Module):
    """ASPP_Block restated (train.py:450-494): aspp1-4 (1x1, dilated 3x3 d=6/12/18) with BN+ReLU,
    image pool (GAP -> 1x1 -> BN -> ReLU -> bilinear-ac back to size), cat, 1x1 1280->256 + BN +
    ReLU."""

    def __init__(self):
        super().__init__()
        self.aspp1 = OracleASPP(256, 256, 1, 0, 1)
        self.aspp2 = OracleASPP(256, 256, 3, 6, 6)
        self.aspp3 = OracleASPP(256, 256, 3, 12, 12)
        self.aspp4 = OracleASPP(256, 256, 3, 18, 18)
        self.global_avg_pool = nn.Sequential(nn.AdaptiveAvgPool2d((1, 1)),
                                             nn.Conv2d(256, 256, 1, bias=False),
                                             nn.BatchNorm2d(256), nn.ReLU())
        self.conv1 = nn.Sequential(nn.Conv2d(1280, 256, 1, bias=False), nn.BatchNorm2d(256),
                                   nn.ReLU())

    def forward(self, x):
        parts = [m(x) for m in (self.aspp1, self.aspp2, self.aspp3, self.aspp4)]
        x5 = F.interpolate(self.global_avg_pool(x), size=x.shape[2:], mode="bilinear",
                           align_corners=True)
        return self.conv1(torch.cat(parts + [x5], dim=1))


class OracleTrainHourglass(nn.Module):
    """hourglass(f) restated (train.py:497-541): stride-2 blocks down, (f -> f/2) blocks on the
    skips and on the way up, ASPP at the bottom, nearest x2 + concat per level."""

    def __init__(self, f):
        super().__init__()
        for i in range(1, 5):
            setattr(self, f"downsample{i}", OracleCmpResidual(f, f, stride=2))
        for i in range(1, 5):
            setattr(self, f"residual{i}", OracleCmpResidual(f, f // 2))
        for i in range(1, 5):
            setattr(self, f"upsample{i}", OracleCmpResidual(f, f // 2))
        self.aspp = OracleTrainASPP()

    def forward(self, x):
        ups, down = [], x
        for i in range(1, 5):
            ups.append(getattr(self, f"residual{i}")(down))
            down = getattr(self, f"downsample{i}")(down)
        out = self.aspp(down)
        for i in range(4, 0, -1):
            out = getattr(self, f"upsample{i}")(F.interpolate(out, scale_factor=2))
            out = torch.cat([out, ups[i - 1]], dim=1)
        return out


class OracleTrainModel(nn.Module):
    """creatModel restated (train.py:543-600): stem 7x7/2 + ReLU + RB(64,128,s2) + RB(128,128) +
    RB(128,f); 3 unshared stages, inter = cat[return(out_k), retuen_2(ll), down_feature(inter)]."""

    def __init__(self, nFeats=256, nOut=(2, 16, 17)):
        super().__init__()
        self.preprocess1 = nn.Sequential(
            nn.Conv2d(3, 64, 7, 2, 3), nn.ReLU(), OracleCmpResidual(64, 128, stride=2),
            OracleCmpResidual(128, 128), OracleCmpResidual(128, nFeats))
        for k in (1, 2):
            setattr(self, f"stage{k}", OracleTrainHourglass(nFeats))
            setattr(self, f"stage{k}_out", nn.Conv2d(nFeats, nOut[k - 1], 1, bias=False))
            setattr(self, f"stage{k}_return", nn.Conv2d(nOut[k - 1], nFeats // 2, 1, bias=False))
            setattr(self, f"stage{k}_retuen_2", nn.Conv2d(nFeats, nFeats // 4, 1, bias=False))
            setattr(self, f"stage{k}_down_feature", nn.Conv2d(nFeats, nFeats // 4, 1, bias=False))
        self.stage3 = OracleTrainHourglass(nFeats)
        self.stage3_out = nn.Conv2d(nFeats, nOut[2], 1, bias=False)

    def forward(self, x):
        inter = self.preprocess1(x)
        out = []
        for k in (1, 2, 3):
            ll = getattr(self, f"stage{k}")(inter)
            tmp = getattr(self, f"stage{k}_out")(ll)
            out.append(tmp)
            if k < 3:
                inter = torch.cat([getattr(self, f"stage{k}_return")(tmp),
                                   getattr(self, f"stage{k}_retuen_2")(ll),
                                   getattr(self, f"stage{k}_down_feature")(inter)], dim=1)
        return out


def bootstrapped_ce(logits, target, fraction):
    """Costomer_CrossEntropyLoss restated (train.py:343-362): per-pixel CE (log-softmax over the
    class axis), the top k = int(h * w * max(fraction, 0.1)) pixels per image, mean."""
    fraction = max(fraction, 0.1)
    loss = F.nll_loss(F.log_softmax(logits, dim=1), target, reduction="none")
    k = int(logits.shape[2] * logits.shape[3] * fraction)
    top, _ = torch.topk(loss.view(logits.shape[0], -1), k)
    return top.mean()


def trainpy_loss(outs, skeleton, keypoints, fraction):
    """train.py:886-890: loss_2 + loss_3, each bootstrapped CE + plain CE (the background head
    out[0] is not in the loss; it still gets gradient through stage1_return)."""
    return (bootstrapped_ce(outs[1], skeleton, fraction) + F.cross_entropy(outs[1], skeleton)
            + bootstrapped_ce(outs[2], keypoints, fraction) + F.cross_entropy(outs[2], keypoints))


def masked_ce(logits, target, mask):
    """Costomer_CrossEntropyLoss_with_mask restated (train.py:365-376): mean of CE * mask."""
    loss = F.nll_loss(F.log_softmax(logits, dim=1), target, reduction="none")
    return (loss * mask.float()).view(loss.shape[0], -1).mean()


def masked_mse(x, target, mask):
    """Costomer_MSELoss_with_mask restated (train.py:379-391): mean of (x - t)^2 * mask[:, None]."""
    loss = F.mse_loss(x, target, reduction="none")
    m = mask.float().view(mask.shape[0], 1, mask.shape[1], mask.shape[2])
    return (loss * m).view(loss.shape[0], -1).mean()


def bootstrapped_mse(x, target, fraction):
    """Costomer_MSELoss restated (train.py:394-408): per image the k = int(h*w*max(f, 0.25))
    largest squared errors over its C*h*w elements, mean."""
    fraction = max(fraction, 0.25)
    loss = F.mse_loss(x, target, reduction="none")
    k = int(x.shape[2] * x.shape[3] * fraction)
    top, _ = torch.topk(loss.view(x.shape[0], -1), k)
    return top.mean()
