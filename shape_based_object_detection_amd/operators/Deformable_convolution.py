"""Drop-in ``operators/Deformable_convolution.py`` (reference :5-146) on the HIP path.

Same module surface: ``DeformConv2d(inc, outc, kernel_size=3, padding=1, stride=1, bias=None,
modulation=True)`` with children ``zero_padding``, ``conv`` (k×k, stride k), ``p_conv`` and
``m_conv`` (3×3, pad 1, stride ``stride``, weights zero-initialised) and the no-op ``_set_lr``
backward hook.  The offset / mask convolutions stay ordinary convolutions (MIOpen); the
sampling + modulation + k×k contraction, forward and backward, is one C-ABI call each
(``sbod_dcn_fwd_f32`` / ``sbod_dcn_bwd_f32``: the forward and the weight gradient as split-bf16
MFMA contractions — each fp32 operand the exact sum of three bf16 parts, six products kept, fp32
accumulation, fp32-level error — and the data gradient on fp32 MFMA) instead of the reference's chain of
gathers, concatenations and an im2col-sized intermediate.  CPU tensors take the host path
(``hostpath.deform_conv2d``: the reference's sampling arithmetic in torch, autograd backward).
"""
import torch
from torch import nn

from .. import core
from .. import hostpath


class DeformConv2d(nn.Module):
    def __init__(self, inc, outc, kernel_size=3, padding=1, stride=1, bias=None, modulation=True):
        super(DeformConv2d, self).__init__()
        self.kernel_size = kernel_size
        self.padding = padding
        self.stride = stride
        self.zero_padding = nn.ZeroPad2d(padding)
        self.conv = nn.Conv2d(inc, outc, kernel_size=kernel_size, stride=kernel_size, bias=bias)

        self.p_conv = nn.Conv2d(inc, 2 * kernel_size * kernel_size, kernel_size=3, padding=1,
                                stride=stride)
        nn.init.constant_(self.p_conv.weight, 0)
        self.p_conv.register_full_backward_hook(self._set_lr)

        self.modulation = modulation
        if modulation:
            self.m_conv = nn.Conv2d(inc, kernel_size * kernel_size, kernel_size=3, padding=1,
                                    stride=stride)
            nn.init.constant_(self.m_conv.weight, 0)
            self.m_conv.register_full_backward_hook(self._set_lr)

    @staticmethod
    def _set_lr(module, grad_input, grad_output):
        # reference :28-31 builds generators and discards them: gradients are left unchanged
        return None

    def forward(self, x):
        offset = self.p_conv(x)
        mask_logits = self.m_conv(x) if self.modulation else None
        if not x.is_cuda:
            out = hostpath.deform_conv2d(x, offset, mask_logits, self.conv.weight, self.kernel_size,
                                         self.padding, self.stride)
            return out + self.conv.bias.view(1, -1, 1, 1) if self.conv.bias is not None else out
        out = core.deform_conv2d(x, offset, mask_logits, self.conv.weight, self.kernel_size,
                                 self.padding, self.stride)
        if self.conv.bias is not None:
            out = out + self.conv.bias.view(1, -1, 1, 1)
        return out
