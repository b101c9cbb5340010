"""bluesky_amd -- MI355X-native BlueSky conflict-detection / propagation hot path.

Drop-ins for the reference's hot path:

* ``bluesky_amd.statebased``  -- ``StateBasedCD.detect`` (CD method module)

All compute runs in the HIP library ``libbsaccel.so`` (gfx950) through the C
ABI in ``include/bsaccel.h``; import works without a GPU, calls raise
``AccelUnavailable`` when the library or a device is missing.
"""
from . import _lib, statebased, synth  # noqa: F401
from ._lib import AccelError, AccelUnavailable, Context, default_context  # noqa: F401

__all__ = ['statebased', 'synth', 'Context', 'default_context', 'AccelError',
           'AccelUnavailable', 'register']


def register(asas_cls=None, cd_name='GPU'):
    """Register the GPU detector as a BlueSky CD method (asas.py:49-51).

    ``asas_cls`` defaults to ``bluesky.traffic.asas.ASAS``; afterwards the
    stack command ``CDMETHOD GPU`` selects it (stack.py:284 -> asas.py:164).
    """
    if asas_cls is None:
        from bluesky.traffic.asas import ASAS as asas_cls  # pragma: no cover
    asas_cls.addCDMethod(cd_name, statebased)
    return asas_cls
