"""Reference module path ``models.RetinaNet`` — the hot-path half: the criterion and the priors.

The network itself (backbone / heads) is out of scope: it runs as ordinary torch convolutions.
"""
from .criteria import RetinaFocalLoss  # noqa: F401
from .priors import priors_cxcy as _priors


def create_anchors(device='cpu'):
    """The constant [P, 4] center-size priors of this architecture (byte-identical to the
    reference generator, see models/priors.py)."""
    return _priors('RETINA', device)
