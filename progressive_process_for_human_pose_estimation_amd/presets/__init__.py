"""Reference model variants on the same HIP engine and kernels.

try_with_aspp   progressive heads (background 2-class CE -> skeleton 20-class CE -> 17 keypoint
                MSE, each re-injected by concat + 1x1), 3 stacks; the hourglass registers the ASPP
                branch but never calls it (try_with_aspp.py:213-279) — BASELINE configs[3].
try_different_stack  the same progressive heads on the primary hourglass (try_different_stack.py).
"""
