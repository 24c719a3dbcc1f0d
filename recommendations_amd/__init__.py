"""recommendations_amd — MI355X (gfx950) native LTHM training hot path.

Drop-in for the hot path of ranjanbalappa-nykaa/recommendations: the modules in
``recommendations_amd.commons`` and ``recommendations_amd.models.lthm`` keep the
reference's class names, constructor signatures, parameter names and
``BaseModelWrapper`` API, while every computation runs in hand-written HIP
kernels (``csrc/``) behind the C ABI declared in ``include/lthm.h``.
"""
__version__ = "0.1.0"
