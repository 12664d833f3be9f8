"""Reference ``models`` package, hot-path half: criteria, priors and detection post-processing.

``model_entry`` of the reference (models/__init__.py:8-32) returns (network, criterion class);
networks are out of scope here, so ``criterion_entry(arch)`` returns the criterion class.
"""
from .criteria import (MultiBoxLoss300, MultiBoxLoss512, RefineDetLoss, RetinaFocalLoss,  # noqa: F401
                       criterion_entry)
from .priors import prior_table, priors_cxcy  # noqa: F401
