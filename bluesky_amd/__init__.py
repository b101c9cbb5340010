"""bluesky_amd -- MI355X-native BlueSky conflict-detection / propagation hot path.

Drop-ins for the reference's hot path:

* ``bluesky_amd.statebased``  -- ``StateBasedCD.detect`` (CD method module)
* ``bluesky_amd.kwik``        -- opt-in flat-earth variant (kwikqdrdist_matrix)

All compute runs in the HIP library ``libbsaccel.so`` (gfx950) through the C
ABI in ``include/bsaccel.h``; import works without a GPU, calls raise
``AccelUnavailable`` when the library or a device is missing.
"""
from . import _lib, dist, kinematics, kwik, mvp, resident, statebased, synth  # noqa: F401
from ._lib import AccelError, AccelUnavailable, Context, default_context  # noqa: F401

__all__ = ['statebased', 'kwik', 'mvp', 'kinematics', 'resident', 'dist', 'synth', 'Context',
           'default_context', 'AccelError', 'AccelUnavailable', 'register']


def register(asas_cls=None, cd_name='GPU', cr_name='GPUMVP', kwik_name='GPUKWIK'):
    """Register the GPU detector and MVP resolver with BlueSky's ASAS.

    ``ASAS.addCDMethod(cd_name, statebased)`` (asas.py:49-51) and
    ``ASAS.addCRMethod(cr_name, mvp)`` (asas.py:53-55); afterwards the stack
    commands ``CDMETHOD GPU`` (stack.py:284 -> asas.py:164) and
    ``RESO GPUMVP`` (stack.py:631 -> asas.py:179) select them.
    ``asas_cls`` defaults to ``bluesky.traffic.asas.ASAS``.
    """
    if asas_cls is None:
        from bluesky.traffic.asas import ASAS as asas_cls  # pragma: no cover
    asas_cls.addCDMethod(cd_name, statebased)
    asas_cls.addCDMethod(kwik_name, kwik)
    asas_cls.addCRMethod(cr_name, mvp)
    return asas_cls
