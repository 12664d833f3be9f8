"""Box codecs of ``dataset/transforms.py:26-83`` on the HIP path (same names and semantics).

The augmentation half of the reference module (expand / random_crop / photometric_distort …)
is CPU data-loader work and out of scope.
"""
from .. import _lib as L
from .. import core


def _rows(t, what):
    L.require_device(t, what=what)
    if t.dim() < 1 or t.shape[-1] != 4:
        raise RuntimeError('%s: expected [..., 4] boxes, got %s' % (what, tuple(t.shape)))
    return t.float()


def xy_to_cxcy(xy):
    """(x_min, y_min, x_max, y_max) -> (c_x, c_y, w, h)  (transforms.py:26-34)."""
    return core.codec('xy_to_cxcy', _rows(xy, 'xy_to_cxcy'))


def cxcy_to_xy(cxcy):
    """(c_x, c_y, w, h) -> (x_min, y_min, x_max, y_max)  (transforms.py:37-45)."""
    return core.codec('cxcy_to_xy', _rows(cxcy, 'cxcy_to_xy'))


def cxcy_to_gcxgcy(cxcy, priors_cxcy):
    """Encode w.r.t. priors: (c - pc) / (pwh / 10), log(wh / pwh) * 5  (transforms.py:48-66)."""
    return core.codec('encode_tenfive', _rows(cxcy, 'cxcy_to_gcxgcy'), priors_cxcy.float())


def gcxgcy_to_cxcy(gcxgcy, priors_cxcy):
    """Decode: g * pwh / 10 + pc, exp(g / 5) * pwh  (transforms.py:69-83)."""
    return core.codec('decode_tenfive', _rows(gcxgcy, 'gcxgcy_to_cxcy'), priors_cxcy.float())
