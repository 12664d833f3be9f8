"""Box codecs of ``dataset/transforms.py:26-83`` (same names and semantics): device tensors run
the HIP kernel (csrc/codec.hip), CPU tensors the host path (``host.py``, the data-loader side).

The augmentation half of the reference module (expand / random_crop / photometric_distort …)
is CPU data-loader work and out of scope.
"""
from .. import _lib as L
from .. import core
from .. import host
from ..metrics import on_host


def _rows(t, what):
    L.require_device(t, what=what)
    if t.dim() < 1 or t.shape[-1] != 4:
        raise RuntimeError('%s: expected [..., 4] boxes, got %s' % (what, tuple(t.shape)))
    return t.float()


def xy_to_cxcy(xy):
    """(x_min, y_min, x_max, y_max) -> (c_x, c_y, w, h)  (transforms.py:26-34)."""
    if on_host(xy):
        return host.xy_to_cxcy(xy)
    return core.codec('xy_to_cxcy', _rows(xy, 'xy_to_cxcy'))


def cxcy_to_xy(cxcy):
    """(c_x, c_y, w, h) -> (x_min, y_min, x_max, y_max)  (transforms.py:37-45)."""
    if on_host(cxcy):
        return host.cxcy_to_xy(cxcy)
    return core.codec('cxcy_to_xy', _rows(cxcy, 'cxcy_to_xy'))


def cxcy_to_gcxgcy(cxcy, priors_cxcy):
    """Encode w.r.t. priors: (c - pc) / (pwh / 10), log(wh / pwh) * 5  (transforms.py:48-66)."""
    if on_host(cxcy, priors_cxcy):
        return host.cxcy_to_gcxgcy(cxcy, priors_cxcy)
    return core.codec('encode_tenfive', _rows(cxcy, 'cxcy_to_gcxgcy'), priors_cxcy.float())


def gcxgcy_to_cxcy(gcxgcy, priors_cxcy):
    """Decode: g * pwh / 10 + pc, exp(g / 5) * pwh  (transforms.py:69-83)."""
    if on_host(gcxgcy, priors_cxcy):
        return host.gcxgcy_to_cxcy(gcxgcy, priors_cxcy)
    return core.codec('decode_tenfive', _rows(gcxgcy, 'gcxgcy_to_cxcy'), priors_cxcy.float())
