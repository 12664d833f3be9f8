"""Reference ``models`` package, hot-path half: criteria, priors and detection post-processing.

``model_entry(config)`` keeps the reference registry's contract (models/__init__.py:8-32): the
arch string of ``config.model['arch']`` selects ``(network, criterion class)``.  The networks
(VGG / ResNet backbones and heads) are out of scope here — they are ordinary torch convolutions
— so the caller registers the network classes it uses, typically the reference's own:

    from shape_based_object_detection_amd import models
    models.register_network('SSD512', reference_models.SSD512.SSD512)
    model, criterion = models.model_entry(config)      # criterion = sbod MultiBoxLoss512

and ``train_anchor.py:172``'s ``criterion(priors_cxcy=model.priors_cxcy, config=config)`` then
builds the HIP criterion.  ``criterion_entry(arch)`` returns the criterion class alone.
"""
from .criteria import (MultiBoxLoss300, MultiBoxLoss512, RefineDetLoss, RetinaFocalLoss,  # noqa: F401
                       criterion_entry)
from .priors import prior_table, priors_cxcy  # noqa: F401

_NETWORKS = {}
# archs whose reference constructor takes (n_classes, device=...) vs (n_classes, config=...)
_DEVICE_ARGS = {'SSD300', 'SSD512'}


def register_network(arch, factory):
    """Network class (or factory) for ``arch`` ('SSD300', 'SSD512', 'RETINA50', 'RETINA101',
    'REFINEDET'), called with the reference's constructor arguments."""
    _NETWORKS[arch.upper()] = factory


def _get(config, key):
    return config[key] if isinstance(config, dict) else getattr(config, key)


def model_entry(config):
    """models/__init__.py:8-32: ``(network, criterion class)`` for ``config.model['arch']``."""
    model = _get(config, 'model')
    arch = str(model['arch']).upper()
    if arch.startswith('FCOS'):
        # the reference's FCOS constructor and loss crash; not rebuilt
        raise NotImplementedError('%s: FCOS is not part of the sbod hot path' % arch)
    crit = criterion_entry(arch)
    factory = _NETWORKS.get(arch)
    if factory is None:
        raise NotImplementedError('model_entry(%s): no network registered — networks are out of scope '
                                  'of sbod; register one with models.register_network(%r, NetworkClass)'
                                  % (arch, arch))
    n_classes = _get(config, 'n_classes')
    if arch in _DEVICE_ARGS:
        net = factory(n_classes, device=_get(config, 'device'))
    else:
        net = factory(n_classes, config=config)
    return net, crit
