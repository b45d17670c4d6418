"""everest_amd — MI355X-native (gfx950) GP-surrogate + qNEHVI hot path of BoFire.

Public surface mirrors BoFire's plugin API for this path:
``everest_amd.strategies.map(data_model)`` / ``everest_amd.surrogates.map(data_model)``.
Dense work runs in hand-written HIP kernels behind the C-ABI in ``include/everest_amd.h``
(``everest_amd/_lib/libeverest_amd.so``); there is no CPU fallback.
"""
__version__ = "0.1.0"
