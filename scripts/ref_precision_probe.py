"""Which side carries the error in the bf16 kernel tests: torch's GPU fp32 conv reference or the
kernel? Both against a float64 CPU conv on the same bf16 operands (small case)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from progressive_process_for_human_pose_estimation_amd import hgk as H  # noqa: E402

torch.backends.cudnn.allow_tf32 = False
torch.backends.cuda.matmul.allow_tf32 = False
L = H.load_library()
g = torch.Generator(device="cuda").manual_seed(11)
N, hw, C = 4, 16, 128
x = (torch.randn(N, hw, hw, C, device="cuda", generator=g) * 0.7).to(torch.bfloat16)
w = torch.randn(C, C, 3, 3, device="cuda", generator=g) * (1.0 / (9 * C) ** 0.5)
bias = torch.randn(C, device="cuda", generator=g) * 0.1
wb = w.to(torch.bfloat16)
a = x.float().permute(0, 3, 1, 2)
ref32 = F.conv2d(a, wb.float(), bias, padding=1)
ref64 = F.conv2d(a.double().cpu(), wb.double().cpu(), bias.double().cpu(), padding=1)
print("torch fp32 GPU conv vs fp64 CPU: max abs err %.3e, max|ref| %.3f" % ((ref32.double().cpu() - ref64).abs().max(), ref64.abs().max()))
ld = L.hgk_conv_w_ld(9 * C)
wp = torch.empty(C, ld, device="cuda", dtype=torch.bfloat16)
H.check(L.hgk_pack_conv_weight(H.stream_handle(), H.BF16, w.data_ptr(), wp.data_ptr(), ld, C, C, 3, 3, 0, C, C))
y = torch.empty(N, hw, hw, C, device="cuda", dtype=torch.bfloat16)
part = torch.empty((2 * (N * hw * hw // 64) + 4) * 3 * C, device="cuda")
rows = H.ctypes.c_int(0)
H.check(L.hgk_conv_fwd(H.stream_handle(), H.BF16, x.data_ptr(), wp.data_ptr(), ld, bias.data_ptr(), None,
                       y.data_ptr(), None, None, 0, 0, part.data_ptr(), H.ctypes.byref(rows), N, hw, hw, C, C,
                       3, 3, 1, 1, 1, None, 0))
torch.cuda.synchronize()
r64 = ref64.permute(0, 2, 3, 1)
e = (y.double().cpu() - r64).abs()
print("kernel (bf16 out) vs fp64: max abs err %.3e; max err / (2^-8 |ref|) %.3f" % (e.max(), (e / (2 ** -8 * r64.abs()).clamp_min(1e-12)).max()))
e32 = (y.double().cpu() - ref32.double().cpu().permute(0, 2, 3, 1)).abs()
print("kernel vs torch fp32 GPU: max abs err %.3e" % e32.max())
bound = 2 ** -8 * r64.abs() + 1e-4 * r64.abs().max()
ratio = e / bound
i = int(ratio.argmax())
print("with abs term: worst ratio %.3f at ref %.5f err %.3e; elements over bound %d of %d" %
      (ratio.max(), r64.reshape(-1)[i], e.reshape(-1)[i], int((ratio > 1).sum()), ratio.numel()))
acc = (r64 - bias.double().cpu()).reshape(-1)[i]
print("  conv part (ref - bias) at that element %.5f, bias %.5f, y %.5f" % (acc, float(bias.double().cpu()[i % C]), float(y.reshape(-1)[i])))
