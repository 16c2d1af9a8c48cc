"""Reference model variants on the same HIP engine and kernels.

try_with_aspp   progressive heads (background 2-class CE -> skeleton 20-class CE -> 17 keypoint
                MSE, each re-injected by concat + 1x1), 3 stacks; the hourglass registers the ASPP
                branch but never calls it (try_with_aspp.py:213-279) — BASELINE configs[3].
try_different_stack  the same progressive heads on the primary hourglass (try_different_stack.py).
try_more_layer  try_with_aspp with the ASPP block LIVE at the innermost level (dilated 3x3s, global
                average pool -> 1x1 -> BN -> ReLU -> broadcast, 1280 -> 256 conv1), 4 stacks.
hourglass_compare  unshared hourglass, always-on BN-ed projection + bn4, nearest up-sampling.
train           stride-2 residual blocks, unshared hourglass with the live ASPP_Block, nearest x2
                + concat, 3 stages (train.py); generateMask.
"""
