"""torch-CPU fp32 restatement of ``operators/Deformable_convolution.py:33-146`` (TEST ONLY).

Sampling semantics restated:
  * offset channels [0, N) move rows, [N, 2N) move columns (N = k²);
  * p = (p_0 + p_n) + offset with p_0 = 1 + idx·stride (the 1 is hard-coded, :103-111) and
    p_n from an ij meshgrid of arange(−(k−1)//2, (k−1)//2 + 1) (:93-101);
  * q_lt = floor(p) from the UNclamped p, q_rb = q_lt + 1, both clamped to the padded map;
    then p itself is clamped (:50-61) — border clamp, never zero outside the padded map;
  * bilinear weights g_* (:64-67), gathered corners summed lt + rb + lb + rt (:76-79),
    times sigmoid modulation (:82-86), then a k×k stride-k bias-free conv (:16, :89).
"""
import torch
import torch.nn.functional as F


def sample_columns(x, offset, mask, ks=3, padding=1, stride=1):
    """Return the modulated sampled tensor [B, C, Ho, Wo, N] (autograd through offset/mask/x)."""
    B, C, H, W = x.shape
    N = ks * ks
    Ho, Wo = offset.shape[2], offset.shape[3]
    xp = F.pad(x, (padding, padding, padding, padding)) if padding else x
    Hp, Wp = xp.shape[2], xp.shape[3]
    r = torch.arange(-(ks - 1) // 2, (ks - 1) // 2 + 1)
    pnx, pny = torch.meshgrid(r, r, indexing='ij')
    pn = torch.cat([pnx.flatten(), pny.flatten()]).view(1, 2 * N, 1, 1).float()
    p0x, p0y = torch.meshgrid(torch.arange(1, Ho * stride + 1, stride),
                              torch.arange(1, Wo * stride + 1, stride), indexing='ij')
    p0 = torch.cat([p0x.flatten().view(1, 1, Ho, Wo).repeat(1, N, 1, 1),
                    p0y.flatten().view(1, 1, Ho, Wo).repeat(1, N, 1, 1)], 1).float()
    p = (p0 + pn + offset).permute(0, 2, 3, 1)            # [B, Ho, Wo, 2N]
    qlt = p.detach().floor()
    qrb = qlt + 1
    lim = lambda t: torch.cat([t[..., :N].clamp(0, Hp - 1), t[..., N:].clamp(0, Wp - 1)], -1)
    qlt, qrb = lim(qlt).long(), lim(qrb).long()
    p = lim(p)
    px, py = p[..., :N], p[..., N:]
    ltx, lty, rbx, rby = qlt[..., :N], qlt[..., N:], qrb[..., :N], qrb[..., N:]
    g_lt = (1 + (ltx.type_as(p) - px)) * (1 + (lty.type_as(p) - py))
    g_rb = (1 - (rbx.type_as(p) - px)) * (1 - (rby.type_as(p) - py))
    g_lb = (1 + (ltx.type_as(p) - px)) * (1 - (rby.type_as(p) - py))
    g_rt = (1 - (rbx.type_as(p) - px)) * (1 + (lty.type_as(p) - py))
    flat = xp.reshape(B, C, Hp * Wp)

    def gat(qx, qy):
        idx = (qx * Wp + qy).reshape(B, 1, -1).expand(B, C, -1)
        return flat.gather(2, idx).view(B, C, Ho, Wo, N)

    xo = (g_lt.unsqueeze(1) * gat(ltx, lty) + g_rb.unsqueeze(1) * gat(rbx, rby)
          + g_lb.unsqueeze(1) * gat(ltx, rby) + g_rt.unsqueeze(1) * gat(rbx, lty))
    if mask is not None:
        xo = xo * mask.permute(0, 2, 3, 1).unsqueeze(1)
    return xo


def deform_conv2d(x, offset, mask, weight, ks=3, padding=1, stride=1):
    """out[b,o,h,w] = Σ_{c,i,j} weight[o,c,i,j] · cols[b,c,h,w,i·k+j]."""
    cols = sample_columns(x, offset, mask, ks, padding, stride)
    B, C, Ho, Wo, N = cols.shape
    return torch.einsum('bchwn,ocn->bohw', cols, weight.reshape(weight.shape[0], C, N))


def deform_module(x, p_w, p_b, m_w, m_b, conv_w, ks=3, padding=1, stride=1):
    """The whole ``DeformConv2d.forward``: offset/mask convs (3×3, pad 1, stride s) + sampling."""
    offset = F.conv2d(x, p_w, p_b, stride=stride, padding=1)
    mask = torch.sigmoid(F.conv2d(x, m_w, m_b, stride=stride, padding=1))
    return deform_conv2d(x, offset, mask, conv_w, ks, padding, stride)
