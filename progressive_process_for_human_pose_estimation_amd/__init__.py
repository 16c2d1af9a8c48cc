"""MI355X-native stacked-hourglass training engine (drop-in for the hot path of
Xinjie-Qiu/progressive_process_for_human_pose_estimation, try_with_torch.py:179-343).

Public surface mirrors the reference: ResidualBlock, hourglass, lin, creatModel (nn.Modules whose
forward/backward run on the libhgk HIP kernels), plus MSELoss (fused HIP per-stack loss) and the
data-parallel Trainer.
"""
from .modules import ResidualBlock, creatModel, hourglass, lin  # noqa: F401

__all__ = ["ResidualBlock", "hourglass", "lin", "creatModel"]
